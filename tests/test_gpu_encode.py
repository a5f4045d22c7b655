""".dt encoding on the GPU side of the engine.

`encode_from(v, ENCODE_FULL)` (src/list/encoding/encode_oplog.rs:404-747, options :122-130) stores
the checkout at `v` in the StartBranch (:606-618); libdtgpu runs that checkout on the device.  The
StartBranch content is the first field appended to the LZ4 buffer, so the decompressed buffer
starts with the device checkout, which must equal the oracle's checkout at `v`.
"""
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog
from test_encoder import _lz4_chunk, _oracle_lz4_decompress

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


@pytest.mark.parametrize("name,frac", [("friendsforever", 0.46), ("git-makefile", 0.3)])
def test_encode_from_full_stores_the_start_branch_checkout(name, frac):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    v = [int(len(o) * frac)]
    full = o.encode_from(v)                      # ENCODE_FULL
    patch = o.encode_from(v, dt_amd.ENCODE_PATCH)
    assert len(full) > len(patch)
    expect = OracleOpLog.load_from(data).checkout_bytes(v)
    ul, block = _lz4_chunk(full)
    raw = _oracle_lz4_decompress(block, ul)
    assert raw[:len(expect)] == expect
    assert raw[:len(expect)] == o.checkout_bytes(v)
    # the patch applies on top of the history at v either way
    for p in (full, patch):
        d = dt_amd.ListOpLog.load_from(o.history(v).encode())
        assert d.decode_and_add(p) == o.local_frontier()
        assert d.checkout_tip_bytes() == o.checkout_tip_bytes()


# ---- the batched device encoder (dt_encoder.hip, dtgpu_batch_encode) ------------------------------
def _unicode_doc(seed):
    o = dt_amd.ListOpLog()
    a, b = o.get_or_create_agent_id("ünï"), o.get_or_create_agent_id("agent-β")
    t1 = o.add_insert(a, 0, "héllo wörld, 日本語のテキスト " * 3)
    o.add_insert_at(b, [t1], 5, "αβγ" * (seed + 1))
    o.add_delete_at(a, [t1], 2, 9)
    o.add_insert(a, 0, "∑ " * 12)
    o.add_delete_without_content(b, 4, 6)
    return o


@pytest.fixture(scope="module")
def corpus():
    docs = [G.dt_bytes(n) for n in G.DT_FILES]
    docs += [dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode() for n in ("sveltecomponent", "friendsforever_flat")]
    docs += [dt_amd.synth_merge_oplog(d, 3000).encode() for d in range(12)]
    docs += [dt_amd.synth_oplog(d, 1500).encode(dt_amd.EncodeOptions(True, False, True)) for d in range(4)]
    docs += [_unicode_doc(s).encode() for s in range(3)]
    with_id = dt_amd.synth_merge_oplog(99, 800)
    with_id.doc_id = "doc-ïd-42"
    docs.append(with_id.encode())
    empty = dt_amd.ListOpLog()
    empty.get_or_create_agent_id("nobody")
    docs.append(empty.encode())
    tiny = dt_amd.ListOpLog()
    tiny.add_insert(tiny.get_or_create_agent_id("seph"), 0, "hi")   # content below the 20-byte LZ4 cut
    docs.append(tiny.encode())
    return docs


@pytest.mark.parametrize("opts", [dt_amd.ENCODE_FULL, dt_amd.EncodeOptions(True, False, True),
                                  dt_amd.EncodeOptions(False, True, True)], ids=["full", "uncompressed", "no_content"])
def test_device_encoder_bytes_equal_host_encoder(corpus, opts):
    b = dt_amd.Batch(docs=corpus, staging="device")
    ms = b.encode(opts)
    assert ms > 0
    for i, d in enumerate(corpus):
        host = dt_amd.ListOpLog.load_from(d).encode(opts)
        assert b.encoded(i) == host, i


def test_device_encoded_files_check_out_to_the_goldens(corpus):
    """Re-encoded on the device, decoded by the oracle: same text as the original (friendsforever
    and the JSON traces: their golden endContent); the LZ4 block decompresses to the walk-order
    text, a permutation of the inserted content."""
    b = dt_amd.Batch(docs=corpus[:5], staging="device")
    b.encode()
    gold = [json_end("friendsforever_flat")] + [None, None] + [json_end("sveltecomponent"), json_end("friendsforever_flat")]
    for i, d in enumerate(corpus[:5]):
        e = b.encoded(i)
        assert e[9] == 5   # CompressedFieldsLZ4 first
        ul, block = _lz4_chunk(e)
        raw = _oracle_lz4_decompress(block, ul)
        assert sorted(raw) == sorted(bytes(dt_amd.ListOpLog.load_from(d).export("content")))
        want = gold[i] if gold[i] is not None else OracleOpLog.load_from(d).checkout_tip_bytes()
        if i != 2:   # node_nodecc: oracle-pinned through the original; the device checks out both
            assert OracleOpLog.load_from(e).checkout_tip_bytes() == want, i
        assert dt_amd.ListOpLog.load_from(e).checkout_tip_bytes() == want, i


def test_device_encoder_reproduces_reference_bytes():
    """The reference-held encoder outputs, byte for byte from the device encoder (not only via the
    host encoder): compat_simple_doc / compat_empty_doc bytes2 (src/list/encoding/tests.rs:374-424)
    from their three older encodings each, and from compat_simple_doc's construction (:396-400)."""
    built = dt_amd.ListOpLog()
    a = built.get_or_create_agent_id("seph")
    built.add_insert(a, 0, "hi there")
    built.add_delete_without_content(a, 3, 7)
    built.add_insert(a, 3, "m")
    srcs = [G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_LZ4, built.encode(),
            G.COMPAT_EMPTY_2, G.COMPAT_EMPTY_1, dt_amd.ListOpLog().encode()]
    want = [bytes(G.COMPAT_SIMPLE_2)] * 4 + [bytes(G.COMPAT_EMPTY_2)] * 3
    b = dt_amd.Batch(docs=[bytes(x) for x in srcs], staging="device")
    b.encode(dt_amd.ENCODE_FULL)
    for i, w in enumerate(want):
        assert b.encoded_status(i) == 0, i
        assert b.encoded(i) == w, i


def json_end(name):
    return G.trace(name)["endContent"].encode()


def test_device_encoder_reports_deferred_documents():
    """A document the batch hands back to the host (DECODE_DEFER: wider than 64 causal chains)
    gets that status from dtgpu_batch_encoded, not bytes."""
    wide = dt_amd.synth_merge_oplog(7, 3000, n_agents=80).encode()
    ok = G.dt_bytes("friendsforever")
    b = dt_amd.Batch(docs=[ok, wide], staging="device")
    b.encode()
    assert b.encoded(0) == dt_amd.ListOpLog.load_from(ok).encode()
    st = b.encoded_status(1)
    if st == 0:   # staged on the device after all: then its bytes must be exact too
        assert b.encoded(1) == dt_amd.ListOpLog.load_from(wide).encode()
    else:
        assert st == 80


def test_device_encoder_random_documents():
    """64 pairwise-merge synthetic documents of varied size and agent count (SURVEY 8(d)4's
    generator), Unicode variants among them, encoded in one batch: every document's bytes equal
    the host encoder's, and the oracle decodes each to the same text as the original."""
    docs = []
    for d in range(64):
        o = dt_amd.synth_merge_oplog(1000 + d, 200 + 97 * d, n_agents=[0, 4, 16, 40][d % 4])
        docs.append(o.encode())
    b = dt_amd.Batch(docs=docs, staging="device")
    b.encode()
    n_dev = 0
    for i, d in enumerate(docs):
        st = b.encoded_status(i)
        if st == 80:   # DECODE_DEFER: wider than the device prep's 64 causal chains
            continue
        assert st == 0, (i, st)
        n_dev += 1
        e = b.encoded(i)
        assert e == dt_amd.ListOpLog.load_from(d).encode(), i
        if i % 8 == 0:
            assert OracleOpLog.load_from(e).checkout_tip_bytes() == OracleOpLog.load_from(d).checkout_tip_bytes(), i
    assert n_dev >= 48


def _round_robin(n_agents, turns, width):
    """A linear history typed by n_agents in turn: one graph entry spanning n_agents * turns agent
    runs (the encoder's sequential agent-run path when that exceeds four)."""
    o = dt_amd.ListOpLog()
    ids = [o.get_or_create_agent_id(f"rr{i}") for i in range(n_agents)]
    pos = 0
    for t in range(turns):
        for a in ids:
            o.add_insert(a, pos, "abcdefgh"[:width])
            pos += width
            if t % 3 == 2:
                o.add_delete_without_content(a, pos - 2, pos - 1)
                pos -= 1
    return o


@pytest.mark.parametrize("n_agents,turns", [(2, 2), (4, 1), (5, 1), (3, 30), (9, 12)])
def test_device_encoder_entries_spanning_many_agent_runs(n_agents, turns):
    docs = [_round_robin(n_agents, turns, w).encode() for w in (1, 3)]
    docs.append(G.dt_bytes("friendsforever"))   # beside a regular document in the same batch
    b = dt_amd.Batch(docs=docs, staging="device")
    b.encode()
    for i, d in enumerate(docs):
        assert b.encoded(i) == dt_amd.ListOpLog.load_from(d).encode(), i
