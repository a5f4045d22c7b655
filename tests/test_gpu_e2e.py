"""Device-staged batches (dtgpu_batch_create_device): `.dt` bytes -> GPU decode -> GPU planner
inputs (dt_prep.hip) -> GPU walk plan -> GPU replay.  Same texts as the host-staged path and
the golden / oracle outputs; the device plan equals the host plan command for command."""
import hashlib

import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _texts(b):
    b.run()
    b.sync()
    res = b.results()
    return res, [b.text(i) if r["status"] == 0 else None for i, r in enumerate(res)]


def test_friendsforever_device_staged():
    want = G.trace("friendsforever_flat")["endContent"].encode()
    b = dt_amd.Batch(docs=[G.dt_bytes("friendsforever")] * 64, staging="device")
    res, texts = _texts(b)
    assert all(r["status"] == 0 for r in res)
    assert all(t == want for t in texts)
    assert b.host_planned() == [0] * 64


@pytest.mark.parametrize("copies", [2048, 10000])
def test_headline_batch_matches_golden(copies):
    """The bench's own path (bench.py defaults: friendsforever x 10,000 device-staged, timed
    passes): every document's (length, hash) equals the golden endContent, on the flat LDS tier
    at full occupancy.  2,048 copies are replayed whole (no cut replay: a batch that fills the
    GPU is left uncut)."""
    want = G.trace("friendsforever_flat")["endContent"].encode()
    h = dt_amd.text_hash(want)
    b = dt_amd.Batch(docs=[G.dt_bytes("friendsforever")] * copies, staging="device")
    b.run()
    b.sync()
    for _ in range(2):
        assert b.run_timed() > 0
    res = b.results()
    bad = [i for i, r in enumerate(res) if r["status"] != 0 or r["text_len"] != len(want) or r["text_hash"] != h]
    assert not bad, f"{len(bad)} documents differ from the golden text, first {bad[:5]}"
    assert b.text(copies - 1) == want
    assert b.host_planned() == [0] * copies
    st = b.doc_stats(copies // 2)
    assert st["lds_index"] == 1 and st["fail_site"] == 0
    if copies == 2048:
        assert all(b.segments(i) == [] for i in range(0, copies, 97))


@pytest.mark.parametrize("name", ["git-makefile", "node_nodecc"])
def test_large_docs_device_staged(name):
    data = G.dt_bytes(name)
    b = dt_amd.Batch(docs=[data], staging="device")
    res, texts = _texts(b)
    # the benchmark files must take the all-device path: a deferral is a regression, not a skip
    assert res[0]["status"] != dt_amd.DECODE_DEFER, "benchmark file deferred to the host"
    assert res[0]["status"] == 0
    assert b.host_planned() == [0]
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    assert hashlib.sha256(texts[0]).hexdigest() == hashlib.sha256(want).hexdigest()


def _hbm_tier_doc():
    """`.dt` bytes of a linear document with ~900k inserted chars: its LDS index estimate
    exceeds the biggest LDS tier (160 KiB), so it replays on the HBM-index tier."""
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("hbm")
    n = 0
    for k in range(9):
        chunk = chr(ord("a") + k) * 100_000
        o.add_insert(a, (k * 7919) % (n + 1), chunk)
        n += len(chunk)
    o.add_delete_without_content(a, 5000, 20_000)
    return o.encode()


@pytest.mark.parametrize("case", ["big_tier_with_error_doc", "big_tier_with_hbm_doc"])
def test_split_pass_joins_big_tier(case):
    """Split pass (a big LDS tier's prep -> plan -> replay on its side stream) with no other
    LDS tier beside it: the main stream must still join the side stream before the HBM tier and
    before the batch counts as done, so results and texts are read after the big tier's replay."""
    if case == "big_tier_with_error_doc":
        docs = [G.dt_bytes("node_nodecc"), b"nope"]
    else:
        docs = [G.dt_bytes("git-makefile"), _hbm_tier_doc()]
    for timed in (False, True):
        b = dt_amd.Batch(docs=docs, staging="device")
        if timed:
            b.run_timed()
            res = b.results()
            texts = [b.text(i) if r["status"] == 0 else None for i, r in enumerate(res)]
        else:
            res, texts = _texts(b)
        assert res[0]["status"] == 0
        want = OracleOpLog.load_from(docs[0]).checkout_tip_bytes()
        assert hashlib.sha256(texts[0]).hexdigest() == hashlib.sha256(want).hexdigest()
        if case == "big_tier_with_error_doc":
            assert res[1]["status"] != 0
        else:
            assert res[1]["status"] == 0 and b.doc_stats(1)["lds_index"] == 0, res[1]
            want1 = OracleOpLog.load_from(docs[1]).checkout_tip_bytes()
            assert texts[1] == want1


def test_prep_bounds_checked_kernel(monkeypatch):
    """Debug mode (device-side bounds asserts): the prep kernel instantiated with an
    assert on every computed table index (child slots, parent-vector rows, chain pairs and
    offsets, dense chain slots, record fields) prepares the benchmark files and synthetic
    concurrent documents with no assert firing, and the checkouts are exact."""
    monkeypatch.setenv("DTGPU_PREP_CHECK", "1")
    docs = [G.dt_bytes(n) for n in G.DT_FILES] + [dt_amd.synth_merge_oplog(i, 3000).encode() for i in range(6)]
    b = dt_amd.Batch(docs=docs, staging="device")
    res, texts = _texts(b)
    assert [r["status"] for r in res] == [0] * len(docs)
    assert b.host_planned() == [0] * len(docs)
    for d, t in zip(docs, texts):
        assert t == OracleOpLog.load_from(d).checkout_tip_bytes()


def test_device_plan_equals_host_plan():
    docs = [G.dt_bytes(n) for n in G.DT_FILES]
    dev = dt_amd.Batch(docs=docs, staging="device")
    host = dt_amd.Batch(docs=docs)
    dev.run(); dev.sync(); host.run(); host.sync()
    assert [r["status"] for r in dev.results()] == [0] * len(docs)
    assert [r["status"] for r in host.results()] == [0] * len(docs)
    assert dev.host_planned() == [0] * len(docs)
    for i in range(len(docs)):
        (dc, dt), (hc, ht) = dev.plan(i), host.plan(i)
        assert np.array_equal(dc, hc), G.DT_FILES[i]
        assert np.array_equal(dt, ht), G.DT_FILES[i]


def test_mixed_errors_and_e2e_rerun():
    good = G.dt_bytes("friendsforever")
    bad = bytearray(good)
    bad[100] ^= 0xFF
    docs = [good, bytes(bad), G.COMPAT_SIMPLE_LZ4, good, b"nope", G.COMPAT_EMPTY_1]
    b = dt_amd.Batch(docs=docs, staging="device")
    h = dt_amd.Batch(docs=docs)
    r1, t1 = _texts(b)
    r2, t2 = _texts(h)
    assert [r["status"] for r in r1] == [r["status"] for r in r2]
    assert t1 == t2
    ms = b.run_e2e_timed()
    assert len(ms) == 4 and all(m > 0 for m in ms)
    r3, t3 = [b.results(), [b.text(i) if r["status"] == 0 else None for i, r in enumerate(b.results())]]
    assert t3 == t1



def test_document_past_the_block_limit():
    """A document of 2.2 M inserted chars: more than the tracker's 65,535 blocks (n_ins / 32 + 2,
    MAX_DOC_BLOCKS: block ids are 16 bits in pc[] and the superblock lists).  It must report a
    status, never a wrong text."""
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("big")
    text = ""
    for k in range(22):
        chunk = chr(ord("a") + k % 26) * 100_000
        pos = (k * 7919) % (len(text) + 1)
        o.add_insert(a, pos, chunk)
        text = text[:pos] + chunk + text[pos:]
    o.add_delete_without_content(a, 1000, 250_000)
    text = text[:1000] + text[250_000:]
    b = dt_amd.Batch(oplogs=[o])
    res, texts = _texts(b)
    assert res[0]["status"] == 65   # DTGPU_ERR_CAPACITY


@pytest.mark.gpu
def test_large_batch_chain_and_walk_kernels():
    """A device-staged batch of 300 documents takes the batch paths: prep as three launches with
    the chain decomposition four documents per wave (chain_kernel), the walk orders four per wave
    (walk_kernel, CSR mode on its own stream beside prep's second half) and the planner's
    lane-parallel phase B.  The pool mixes friendsforever (golden, 4 causal chains),
    pairwise-merge documents of 4-16 agents (9-33 chains: past chain_kernel's 16, prep's second
    half redoes the decomposition) and 40-agent ones (64-69 chains: 64 plans on the device, the
    wider ones go through the host-staged retry).  Every text equals the golden / oracle text,
    with the walk overlapped and serialised."""
    import os
    pool = [G.dt_bytes("friendsforever")]
    pool += [dt_amd.synth_merge_oplog(d, 1200 + 60 * d).encode() for d in range(12)]
    pool += [dt_amd.synth_merge_oplog(100 + d, 2000, 40).encode() for d in range(4)]
    want = [G.trace("friendsforever_flat")["endContent"].encode()]
    want += [OracleOpLog.load_from(x).checkout_tip_bytes() for x in pool[1:]]
    docs = [pool[i % len(pool)] for i in range(300)]
    b = dt_amd.Batch(docs=docs, staging="device")
    for overlap in (True, False):
        if not overlap:
            os.environ["DTGPU_NO_WALK_OVERLAP"] = "1"
        try:
            b.run()
            b.sync()
        finally:
            os.environ.pop("DTGPU_NO_WALK_OVERLAP", None)
        res = b.results()
        assert all(r["status"] == 0 for r in res)
        bad = [i for i in range(len(docs)) if b.text(i) != want[i % len(pool)]]
        assert not bad, (overlap, bad[:10])
