"""`ListOpLog::decode_and_add` (src/list/encoding/decode_oplog.rs:465-583, overlap filter
:670-913): merging a `.dt` file or patch into an oplog that already holds operations (host code,
csrc/dt_host.cpp::decode_into / decode_and_add, C ABI dtgpu_oplog_decode_and_add).

The reference's own tests of this path (src/list/encoding/tests.rs:36-372) are restated first,
with the same documents, calls and expected results; oplog equality (`assert_eq!(oplog, ..)`) is
checked on the exported SoA arrays.  Then properties on the benchmark files: a history split at
random versions and re-merged (catch-up path and overlap path, in both orders) holds the same
operations keyed by (agent, seq) as the whole file, re-adding a file changes nothing, and the C
oracle checks out the merged oplog's encoding to the same text as the original file.  GPU tests
check the merged oplog out on the device against the oracle.
"""
import random

import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog
from test_encoder import VECTORS, _keyed
import dt_amd

BaseVersionUnknown, DocIdMismatch, ChecksumFailed = 4, 3, 18


def _names(o):
    return [n.decode() if isinstance(n, bytes) else n for n in o.export("agent_names")]


def _state(o):
    """What `ListOpLog: PartialEq` compares (src/list/eq.rs:21-189), independent of LV order: the
    doc id, each op keyed by (agent name, seq) with its kind, position, content and parents, the
    frontier as (agent, seq) ids, and each agent's next seq."""
    names = _names(o)
    av = {}
    for lv, ln, agent, seq in np.asarray(o.export("agent_runs")).reshape(-1, 4):
        for k in range(int(ln)):
            av[int(lv) + k] = (names[int(agent)], int(seq) + k)
    next_seq = {}
    for (name, seq) in av.values():
        next_seq[name] = max(next_seq.get(name, 0), seq + 1)
    return {"doc_id": o.doc_id, "ops": _keyed(o), "frontier": sorted(av[v] for v in o.local_frontier()),
            "next_seq": next_seq}


def _exact(o):
    """The oplog's arrays exactly as stored (same LV order), for unwinding checks."""
    out = {"names": _names(o), "version": o.local_frontier(), "doc_id": o.doc_id}
    for what in ("ops", "agent_runs", "entries", "parent_offsets", "parents", "content", "char_offsets"):
        out[what] = np.asarray(o.export(what)).tolist()
    return out


def _simple_doc():
    """tests.rs:7-15: "hi there", delete 3..7, insert "m" at 3 -> "hi me"."""
    o = dt_amd.ListOpLog()
    o.get_or_create_agent_id("seph")
    o.add_insert(0, 0, "hi there")
    o.add_delete_without_content(0, 3, 7)
    o.add_insert(0, 3, "m")
    return o


def _clone(o):
    c = dt_amd.ListOpLog()
    if len(o) or o.doc_id is not None:
        c.decode_and_add(o.encode())
    return c


def _err(fn):
    with pytest.raises(dt_amd.ParseError) as e:
        fn()
    return e.value.code


# ---- the reference's tests (src/list/encoding/tests.rs) -------------------------------------

def test_encode_decode_smoke():   # :35-47
    doc = _simple_doc()
    assert _state(dt_amd.ListOpLog.load_from(doc.encode())) == _state(doc)


def test_decode_in_parts():   # :49-74
    doc = dt_amd.ListOpLog()
    doc.get_or_create_agent_id("seph")
    doc.get_or_create_agent_id("mike")
    doc.add_insert(0, 0, "hi there")
    data_1 = doc.encode()
    f1 = doc.local_frontier()
    doc.add_delete_without_content(1, 3, 7)
    doc.add_insert(0, 3, "m")
    f2 = doc.local_frontier()
    data_2 = doc.encode_from(f1, dt_amd.ENCODE_PATCH)

    d2 = dt_amd.ListOpLog()
    assert d2.decode_and_add(data_1) == f1
    assert d2.decode_and_add(data_2) == f2
    assert _state(d2) == _state(doc)


def test_merge_parts():   # :76-90
    oplog = dt_amd.ListOpLog()
    oplog.get_or_create_agent_id("seph")
    oplog.add_insert(0, 0, "hi")
    data_1 = oplog.encode()
    oplog.add_insert(0, 2, " there")
    data_2 = oplog.encode()
    log2 = dt_amd.ListOpLog.load_from(data_1)
    final_v = log2.decode_and_add(data_2)   # overlaps: "hi" is already here
    assert _state(log2) == _state(oplog)
    assert final_v == oplog.local_frontier()


def test_merge_future_patch_errors():   # :92-101
    oplog = _simple_doc()
    v = oplog.local_frontier()[0]
    data = oplog.encode_from([v - 1], dt_amd.ENCODE_PATCH)
    assert _err(lambda: dt_amd.ListOpLog.load_from(data)) == BaseVersionUnknown


def test_merge_parts_2():   # :103-130 (#[ignore] in the reference: b before a names an unknown base)
    oplog_a = dt_amd.ListOpLog()
    oplog_a.get_or_create_agent_id("a")
    oplog_a.get_or_create_agent_id("b")
    t1 = oplog_a.add_insert(0, 0, "aa")
    data_a = oplog_a.encode()
    oplog_a.add_insert_at(1, [], 0, "bbb")
    data_b = oplog_a.encode_from([t1], dt_amd.ENCODE_PATCH)

    a_then_b = dt_amd.ListOpLog()
    a_then_b.decode_and_add(data_a)
    a_then_b.decode_and_add(data_b)
    assert _state(a_then_b) == _state(oplog_a)

    b_then_a = dt_amd.ListOpLog()
    assert _err(lambda: b_then_a.decode_and_add(data_b)) == BaseVersionUnknown   # "errors (arguably correctly)"
    assert len(b_then_a) == 0 and _names(b_then_a) == []


def test_encode_reordered_and_shared_agent():   # :141-166
    for names in (("seph", "mike"), ("seph",)):
        oplog = dt_amd.ListOpLog()
        for n in names:
            oplog.get_or_create_agent_id(n)
        a = oplog.add_insert_at(0, [], 0, "a")
        oplog.add_insert_at(len(names) - 1, [], 0, "b")
        oplog.add_insert_at(0, [a], 1, "c")
        assert _state(dt_amd.ListOpLog.load_from(oplog.encode())) == _state(oplog)


def _check_unroll_works(dest, src):   # :180-228
    """Every single-byte corruption of src's encoding, added to a copy of dest: an error leaves the
    copy equal to dest, a success makes it equal to src."""
    enc = src.encode()
    dest_bytes = dest.encode() if len(dest) else None
    fresh = lambda: dt_amd.ListOpLog.load_from(dest_bytes) if dest_bytes else dt_amd.ListOpLog()
    want_dest, want_src = _exact(fresh()), _state(src)
    n_err = 0
    for i in range(len(enc)):
        bad = bytearray(enc)
        bad[i] ^= 0xFF
        out = fresh()
        try:
            out.decode_and_add(bytes(bad))
        except dt_amd.ParseError:
            n_err += 1
            assert _exact(out) == want_dest, i   # unwound exactly
        else:
            assert _state(out) == want_src, i
    return n_err


def test_error_unrolling():   # :230-235
    assert _check_unroll_works(dt_amd.ListOpLog(), _simple_doc()) > 0


def test_error_unrolling_into_non_empty_oplog():
    """The same, merging into an oplog that already holds a prefix of the document (both the
    catch-up and the overlap path unwind)."""
    src = _simple_doc()
    prefix = src.history([3])
    assert len(prefix) == 4
    assert _check_unroll_works(prefix, src) > 0


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_failed_merge_unwinds_runs_extended_in_place(name):
    """A whole benchmark file with a bad checksum merged on top of a prefix of itself: the decode
    appends every operation (extending the prefix's last op / agent / graph runs in place) before
    the checksum fails, and the truncating unwind restores the prefix exactly; the good file then
    merges as if the failed call never happened (the per-agent seq maps were unwound too)."""
    data = G.dt_bytes(name)
    full = dt_amd.ListOpLog.load_from(data)
    want = _keyed(full)
    v = full.dominators([len(full) // 3])
    d = dt_amd.ListOpLog.load_from(full.history(v).encode())
    before = _exact(d)
    bad = bytearray(data)
    bad[-1] ^= 0xFF
    assert _err(lambda: d.decode_and_add(bytes(bad))) == ChecksumFailed
    assert _exact(d) == before
    assert d.decode_and_add(data) == d.local_frontier()
    assert _keyed(d) == want


def test_save_load_save_load():   # :237-268 (content not stored)
    o2 = dt_amd.ListOpLog.load_from(_simple_doc().encode(dt_amd.EncodeOptions(False, True, True)))
    o3 = dt_amd.ListOpLog.load_from(o2.encode(dt_amd.EncodeOptions(False, True, True)))
    assert _state(o2) == _state(o3)


def test_doc_id_preserved():   # :270-281
    oplog = _simple_doc()
    oplog.doc_id = "hi"
    result = dt_amd.ListOpLog.load_from(oplog.encode())
    assert _state(result) == _state(oplog)
    assert result.doc_id == "hi"


def test_mismatched_doc_id_errors():   # :283-293
    o1 = _simple_doc()
    o1.doc_id = "aaa"
    o2 = _simple_doc()
    o2.doc_id = "bbb"
    before = _exact(o2)
    assert _err(lambda: o2.decode_and_add(o1.encode())) == DocIdMismatch
    assert o2.doc_id == "bbb"
    assert _exact(o2) == before


def test_doc_id_preserved_when_error_happens():   # :295-310
    o1 = dt_amd.ListOpLog()
    o2 = _simple_doc()
    o2.doc_id = "bbb"
    data = bytearray(o2.encode())
    data[-1] ^= 0xFF
    assert _err(lambda: o1.decode_and_add(bytes(data))) == ChecksumFailed
    assert o1.doc_id is None and len(o1) == 0


def test_merge_returns_root_for_empty_file():   # :312-320
    assert dt_amd.ListOpLog().decode_and_add(dt_amd.ListOpLog().encode()) == []


def test_merge_returns_version_even_with_overlap():   # :322-331
    oplog = _simple_doc()
    o2 = _clone(oplog)
    assert o2.decode_and_add(oplog.encode()) == o2.local_frontier()


def test_merge_patch_returns_correct_version():   # :333-348
    oplog = _simple_doc()
    v = oplog.local_frontier()
    o2 = _clone(oplog)
    oplog.add_insert(0, 0, "x")
    assert o2.decode_and_add(oplog.encode_from(v, dt_amd.ENCODE_PATCH)) == o2.local_frontier()
    assert _state(o2) == _state(oplog)


def test_regression_1():   # :359-372
    doc = bytes(VECTORS["regression_1.doc_data"])
    patch = bytes(VECTORS["regression_1.patch_data"])
    o = dt_amd.ListOpLog.load_from(doc)
    base = _keyed(o)
    n0 = len(o)
    o.decode_and_add(patch)
    merged = _keyed(o)
    # the patch names a base the document has; what it carries overlaps the document's ops
    assert len(o) >= n0 and all(merged[k] == v for k, v in base.items())
    # the merged oplog round-trips, and the oracle checks out its encoding like the original
    again = dt_amd.ListOpLog.load_from(o.encode())
    assert _keyed(again) == merged
    OracleOpLog.load_from(o.encode()).checkout_tip_bytes()


# ---- properties on the benchmark files -----------------------------------------------------

def _split_versions(o, rng, k):
    n = len(o)
    return [o.dominators([v]) for v in sorted(rng.sample(range(1, n - 1), k))]


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_catch_up_and_overlap_merges_rebuild_the_file(name):
    data = G.dt_bytes(name)
    full = dt_amd.ListOpLog.load_from(data)
    want = _keyed(full)
    rng = random.Random(5)
    for v in _split_versions(full, rng, 2):
        part = full.history(v).encode()
        # catch-up: the patch starts at the part's version (no filtering)
        d = dt_amd.ListOpLog.load_from(part)
        assert d.decode_and_add(full.encode_from(v, dt_amd.ENCODE_PATCH)) == d.local_frontier()
        assert _keyed(d) == want, v
        # overlap: the whole file on top of the part (the part's operations are filtered out)
        d = dt_amd.ListOpLog.load_from(part)
        assert d.decode_and_add(data) == d.local_frontier()
        assert len(d) == len(full) and _keyed(d) == want, v


def test_concurrent_histories_merge_in_either_order():
    """Hist(v1) + Hist(v2) of two concurrent friendsforever versions, merged both ways: the same
    operations as Hist(v1 u v2), and the same text in the oracle."""
    full = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    ora = OracleOpLog.load_from(G.dt_bytes("friendsforever"))
    rng = random.Random(9)
    done = 0
    while done < 3:
        v1, v2 = _split_versions(full, rng, 2)
        u = full.dominators(v1, v2)
        if u in (v1, v2):
            continue   # not concurrent
        h1, h2 = full.history(v1).encode(), full.history(v2).encode()
        want = _keyed(full.history(u))
        texts = []
        for a, b in ((h1, h2), (h2, h1)):
            d = dt_amd.ListOpLog.load_from(a)
            d.decode_and_add(b)
            assert _keyed(d) == want
            texts.append(OracleOpLog.load_from(d.encode()).checkout_tip_bytes())
        assert texts[0] == texts[1] == ora.checkout_bytes(u)
        done += 1


@pytest.mark.parametrize("name", G.DT_FILES)
def test_re_adding_a_file_changes_nothing(name):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    before = _exact(o)
    assert o.decode_and_add(data) == before["version"]
    assert _exact(o) == before


def test_merged_encoding_checks_out_like_the_file():
    """The oracle's checkout of the re-merged oplog's encoding equals its checkout of the file."""
    data = G.dt_bytes("friendsforever")
    full = dt_amd.ListOpLog.load_from(data)
    v = full.dominators([len(full) // 2])
    d = dt_amd.ListOpLog.load_from(full.history(v).encode())
    d.decode_and_add(data)
    assert OracleOpLog.load_from(d.encode()).checkout_tip_bytes() == OracleOpLog.load_from(data).checkout_tip_bytes()


# ---- GPU -----------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_gpu_checkout_of_merged_oplog(name):
    data = G.dt_bytes(name)
    full = dt_amd.ListOpLog.load_from(data)
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    rng = random.Random(21)
    for v in _split_versions(full, rng, 2):
        d = dt_amd.ListOpLog.load_from(full.history(v).encode())
        d.decode_and_add(data)   # overlap path: LVs in a different order from the file's
        assert d.checkout_tip_bytes() == want, v


@pytest.mark.gpu
def test_gpu_checkout_of_concurrent_merge():
    full = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    ora = OracleOpLog.load_from(G.dt_bytes("friendsforever"))
    rng = random.Random(23)
    done = 0
    while done < 2:
        v1, v2 = _split_versions(full, rng, 2)
        u = full.dominators(v1, v2)
        if u in (v1, v2):
            continue
        d = dt_amd.ListOpLog.load_from(full.history(v2).encode())
        d.decode_and_add(full.history(v1).encode())
        assert d.checkout_tip_bytes() == ora.checkout_bytes(u)
        done += 1


def test_doc_id_export_matches_the_oplog():
    """DTGPU_EXPORT_DOC_ID (the array the device decode_and_add tests compare): a presence byte,
    then the id's bytes."""
    o = _simple_doc()
    assert bytes(o.export("doc_id")) == b"\x00"
    o.doc_id = "hi"
    assert bytes(o.export("doc_id")) == b"\x01hi"
    assert bytes(dt_amd.ListOpLog.load_from(o.encode()).export("doc_id")) == b"\x01hi"


def test_device_decode_add_rejects_bad_arguments():
    """dtgpu_decode_add / dtgpu_decode_add_result validate their handles before any device work."""
    import ctypes
    L = dt_amd.lib()
    out = ctypes.c_void_p()
    assert L.dtgpu_decode_add(None, None, None, 0, 0, None, ctypes.byref(out)) == 67   # DTGPU_ERR_ARG
    assert L.dtgpu_decode_add_result(None, 0, None, 0, None) == 67
    assert L.dtgpu_batch_create_decoded(None, ctypes.byref(out)) == 67
