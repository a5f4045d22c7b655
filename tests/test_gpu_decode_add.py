"""`ListOpLog::decode_and_add` on the GPU (dtgpu_decode_add, dt_decode.hip decode_add_kernel):
a batch of (resident oplog, patch) pairs merged by one wavefront each.

The host decode_and_add (csrc/dt_host.cpp, pinned by the reference's own tests in
tests/test_decode_and_add.py, src/list/encoding/tests.rs:36-372) is the checker: for every case the
device's merged arrays equal the host oplog's element for element (same LV order, same RLE runs),
the status and the returned version are the same, and a failed merge leaves the resident document
exactly as it was.  The merged batch then checks out on the device against the oracle."""
import random

import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog
from test_encoder import VECTORS
import dt_amd

pytestmark = pytest.mark.gpu

ARRAYS = ("ops", "agent_runs", "entries", "parent_offsets", "parents", "content", "char_offsets", "version")


def _host_exact(o):
    out = {"names": [bytes(n) for n in o.export("agent_names")], "doc_id": o.doc_id}
    for what in ARRAYS:
        out[what] = np.asarray(o.export(what)).tolist()
    return out


def _dev_exact(m, i):
    out = {"names": [bytes(n) for n in m.export(i, "agent_names")], "doc_id": m.doc_id(i)}
    for what in ARRAYS:
        out[what] = np.asarray(m.export(i, what)).tolist()
    return out


def _host_add(base, patch):
    """(status, frontier, merged host oplog) of the host decode_and_add."""
    o = dt_amd.ListOpLog.load_from(base) if base is not None else dt_amd.ListOpLog()
    try:
        f = o.decode_and_add(patch)
        return 0, f, o
    except dt_amd.ParseError as e:
        return e.code, [], o


def _check_batch(pairs):
    """Merge every (base bytes, patch bytes) pair on the device in one batch; compare with the host.
    Returns the merged DecodeBatch and the device statuses."""
    empty = dt_amd.ListOpLog().encode()
    bases = [b if b is not None else empty for b, _ in pairs]
    d = dt_amd.DecodeBatch(bases)
    d.run()
    for i in range(len(bases)):
        assert d.status(i)["status"] == 0, i
    m = d.add([p for _, p in pairs])
    sts = []
    for i, (b, p) in enumerate(pairs):
        st, f = m.add_result(i)
        sts.append(st)
        if st == dt_amd.DECODE_DEFER:
            continue   # handed to the host path (positions or seqs >= 2^31 and the like)
        hst, hf, ho = _host_add(b, p)
        assert st == hst, (i, st, hst)
        assert _dev_exact(m, i) == _host_exact(ho), i
        if st == 0:
            assert sorted(f) == sorted(hf), i
    return m, sts


def _simple_doc():
    o = dt_amd.ListOpLog()
    o.get_or_create_agent_id("seph")
    o.add_insert(0, 0, "hi there")
    o.add_delete_without_content(0, 3, 7)
    o.add_insert(0, 3, "m")
    return o


def test_reference_cases():
    """tests.rs decode_in_parts, merge_parts, merge_parts_2 (both orders), merge patch version,
    overlap version, regression_1, empty file: one batch, every case equal to the host."""
    pairs = []
    doc = dt_amd.ListOpLog()
    doc.get_or_create_agent_id("seph")
    doc.get_or_create_agent_id("mike")
    doc.add_insert(0, 0, "hi there")
    data_1 = doc.encode()
    f1 = doc.local_frontier()
    doc.add_delete_without_content(1, 3, 7)
    doc.add_insert(0, 3, "m")
    pairs += [(None, data_1), (data_1, doc.encode_from(f1, dt_amd.ENCODE_PATCH))]   # decode_in_parts

    o = dt_amd.ListOpLog()
    o.get_or_create_agent_id("seph")
    o.add_insert(0, 0, "hi")
    d1 = o.encode()
    o.add_insert(0, 2, " there")
    pairs.append((d1, o.encode()))   # merge_parts: overlap

    a = dt_amd.ListOpLog()
    a.get_or_create_agent_id("a")
    a.get_or_create_agent_id("b")
    t1 = a.add_insert(0, 0, "aa")
    da = a.encode()
    a.add_insert_at(1, [], 0, "bbb")
    db = a.encode_from([t1], dt_amd.ENCODE_PATCH)
    pairs += [(da, db), (None, db)]   # merge_parts_2: a then b; b first names an unknown base

    s = _simple_doc()
    v = s.local_frontier()
    sd = s.encode()
    s.add_insert(0, 0, "x")
    pairs += [(sd, s.encode_from(v, dt_amd.ENCODE_PATCH)), (sd, sd)]   # patch version; overlap version
    pairs.append((bytes(VECTORS["regression_1.doc_data"]), bytes(VECTORS["regression_1.patch_data"])))
    pairs.append((None, dt_amd.ListOpLog().encode()))
    _, sts = _check_batch(pairs)
    assert sts[4] == 4 and sts[:4] == [0, 0, 0, 0] and all(x == 0 for x in sts[5:]), sts


def test_doc_ids():
    """tests.rs:270-310: a doc id is kept, a different one on a non-empty oplog is DocIdMismatch
    (the resident document unchanged), and a failing file does not set it."""
    o1 = _simple_doc()
    o1.doc_id = "aaa"
    o2 = _simple_doc()
    o2.doc_id = "bbb"
    bad = bytearray(o2.encode())
    bad[-1] ^= 0xFF
    m, sts = _check_batch([(o2.encode(), o1.encode()), (None, o1.encode()), (None, bytes(bad)),
                           (o2.encode(), o2.encode())])
    assert sts == [3, 0, 18, 0]
    assert m.doc_id(0) == "bbb" and m.doc_id(1) == "aaa" and m.doc_id(2) is None


@pytest.mark.parametrize("prefix", [False, True])
def test_every_corruption_unwinds_like_the_host(prefix):
    """tests.rs:180-235 check_unroll_works: every single-byte corruption of a document's encoding
    merged into an empty oplog, or into a prefix of the document (catch-up and overlap paths):
    the device status equals the host's, and the merged arrays equal the host oplog's -- the
    resident document itself after an error."""
    src = _simple_doc()
    base = src.history([3]).encode() if prefix else None
    enc = src.encode()
    pairs = []
    for i in range(len(enc)):
        bad = bytearray(enc)
        bad[i] ^= 0xFF
        pairs.append((base, bytes(bad)))
    _, sts = _check_batch(pairs)
    assert sum(1 for s in sts if s not in (0, dt_amd.DECODE_DEFER)) > len(enc) // 2


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_benchmark_files_split_and_re_merged(name):
    """A benchmark history split at random versions: the part plus the patch after it
    (catch-up), the part plus the whole file (overlap), the whole file plus itself, and the
    whole file plus a patch it already holds -- in one batch, each equal to the host."""
    data = G.dt_bytes(name)
    full = dt_amd.ListOpLog.load_from(data)
    rng = random.Random(5)
    pairs = []
    for v in [full.dominators([x]) for x in sorted(rng.sample(range(1, len(full) - 1), 3))]:
        part = full.history(v).encode()
        pairs += [(part, full.encode_from(v, dt_amd.ENCODE_PATCH)), (part, data), (data, full.encode_from(v, dt_amd.ENCODE_PATCH))]
    pairs.append((data, data))
    _, sts = _check_batch(pairs)
    assert all(s == 0 for s in sts), sts


def test_concurrent_histories_checkout_on_the_device():
    """Hist(v1) + Hist(v2) of concurrent friendsforever versions merged on the device in both
    orders, then checked out on the device: the oracle's text at v1 u v2."""
    data = G.dt_bytes("friendsforever")
    full = dt_amd.ListOpLog.load_from(data)
    ora = OracleOpLog.load_from(data)
    rng = random.Random(9)
    pairs, want = [], []
    while len(pairs) < 6:
        x1, x2 = sorted(rng.sample(range(1, len(full) - 1), 2))
        v1, v2 = full.dominators([x1]), full.dominators([x2])
        u = full.dominators(v1, v2)
        if u in (v1, v2):
            continue
        h1, h2 = full.history(v1).encode(), full.history(v2).encode()
        pairs += [(h1, h2), (h2, h1)]
        t = ora.checkout_bytes(u)
        want += [t, t]
    m, sts = _check_batch(pairs)
    assert all(s == 0 for s in sts)
    b = m.checkout_batch()
    b.run()
    for i, t in enumerate(want):
        assert b.text(i) == t, i


def test_merged_benchmark_files_check_out():
    """Every benchmark file rebuilt on the device from a prefix plus the file (overlap path) checks
    out on the device to the oracle's text of the file."""
    pairs, want = [], []
    for name in G.DT_FILES:
        data = G.dt_bytes(name)
        full = dt_amd.ListOpLog.load_from(data)
        v = full.dominators([len(full) // 2])
        pairs.append((full.history(v).encode(), data))
        want.append(OracleOpLog.load_from(data).checkout_tip_bytes())
    d = dt_amd.DecodeBatch([p for p, _ in pairs])
    d.run()
    m = d.add([x for _, x in pairs])
    assert [m.add_result(i)[0] for i in range(len(pairs))] == [0] * len(pairs)
    b = m.checkout_batch()
    b.run()
    for i, t in enumerate(want):
        assert b.text(i) == t, i


def test_chained_merges_rebuild_the_history():
    """A history delivered as a chain of patches (encode_from at increasing versions), each merged
    into the previous merge's output on the device -- the merged handle is the next base --
    for several random version chains at once: every link equals the host's oplog after the same
    sequence of decode_and_add calls, and the last one checks out to the oracle's text."""
    data = G.dt_bytes("friendsforever")
    full = dt_amd.ListOpLog.load_from(data)
    ora = OracleOpLog.load_from(data)
    rng = random.Random(13)
    chains = []
    for _ in range(4):
        vs = [full.dominators([x]) for x in sorted(rng.sample(range(1, len(full) - 1), 4))] + [full.local_frontier()]
        parts = [full.history(vs[0]).encode()]
        parts += [full.history(b).encode_from(a, dt_amd.ENCODE_PATCH) for a, b in zip(vs, vs[1:])]
        chains.append((vs, parts))
    hosts = [dt_amd.ListOpLog.load_from(parts[0]) for _, parts in chains]
    d = dt_amd.DecodeBatch([parts[0] for _, parts in chains])
    d.run()
    cur = d
    for k in range(1, 5):
        m = cur.add([parts[k] for _, parts in chains])
        for i, (vs, parts) in enumerate(chains):
            st, f = m.add_result(i)
            hf = hosts[i].decode_and_add(parts[k])
            assert st == 0 and sorted(f) == sorted(hf), (i, k)
            assert _dev_exact(m, i) == _host_exact(hosts[i]), (i, k)
        cur = m
    b = cur.checkout_batch()
    b.run()
    want = ora.checkout_tip_bytes()
    for i in range(len(chains)):
        assert b.text(i) == want, i


def test_random_split_merges_in_random_order():
    """Hist(v) parts of a git-makefile history at random versions merged into each other in
    random order (overlap filter everywhere): statuses and arrays equal the host's."""
    data = G.dt_bytes("git-makefile")
    full = dt_amd.ListOpLog.load_from(data)
    rng = random.Random(17)
    pairs = []
    for _ in range(8):
        a, b = (full.dominators([x]) for x in rng.sample(range(1, len(full) - 1), 2))
        pairs.append((full.history(a).encode(), full.history(b).encode()))
    _, sts = _check_batch(pairs)
    assert all(s == 0 for s in sts), sts
