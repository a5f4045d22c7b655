"""Cut replay (dt_replay.hip "segments"): a long document replays as LV segments on separate
waves -- cut where everything below the cut is one version that every later op has seen, the
boundary the reference fast-forwards across (src/listmerge/merge.rs:811-840) -- each later
segment starting from placeholders for the text at its cut, and the combine step joins the
segments' source lists into the text.  Every text must equal the golden / oracle text, with
segmenting forced onto documents that would replay whole by default, through both staging
paths, the timed pass, the debug invariant checks and the LDS -> HBM tier hand-back."""
import hashlib

import pytest

import golden_data as G
from synth_docs import phased_doc
from oracle.oracle import OpLog as OracleOpLog

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _run(docs, staging, timed=False):
    b = dt_amd.Batch(docs=docs, staging=staging)
    if timed:
        b.run_timed()
    else:
        b.run()
        b.sync()
    res = b.results()
    return b, res, [b.text(i) if r["status"] == 0 else None for i, r in enumerate(res)]


def _check_segments(segs, min_count=2):
    assert len(segs) >= min_count, segs
    assert segs[0]["lo"] == 0 and segs[-1]["hi"] == 0xFFFFFFFF
    for a, b in zip(segs, segs[1:]):
        assert a["hi"] == b["lo"] and a["lo"] < a["hi"]
    assert all(s["status"] == 0 for s in segs), segs
    # the ranges the pass used are the device cut planning's own (cut_kernel), equal to the host
    # plan staging reserved the arenas from; the host-plan fallback never engaged
    for s in segs:
        assert s["host_fallback"] == 0, segs
        assert (s["lo"], s["hi"], s["placeholders"]) == (s["host_lo"], s["host_hi"], s["host_placeholders"]), segs


FF_WANT = None


def _ff_want():
    global FF_WANT
    if FF_WANT is None:
        FF_WANT = G.trace("friendsforever_flat")["endContent"].encode()
    return FF_WANT


@pytest.mark.parametrize("staging", ["device", "host"])
def test_forced_segments_friendsforever(monkeypatch, staging):
    monkeypatch.setenv("DTGPU_SEG_OPS", "300")
    b, res, texts = _run([G.dt_bytes("friendsforever")] * 3, staging)
    assert [r["status"] for r in res] == [0, 0, 0]
    assert all(t == _ff_want() for t in texts)
    for i in range(3):
        _check_segments(b.segments(i), 4)


def test_forced_segments_timed_and_rerun(monkeypatch):
    monkeypatch.setenv("DTGPU_SEG_OPS", "500")
    b = dt_amd.Batch(docs=[G.dt_bytes("friendsforever")] * 2, staging="device")
    for _ in range(2):   # a rerun replays every segment and combines again from scratch
        b.run_timed()
        res = b.results()
        assert [r["status"] for r in res] == [0, 0]
        assert all(b.text(i) == _ff_want() for i in range(2))
    _check_segments(b.segments(0))


def test_node_nodecc_segments_by_default():
    data = G.dt_bytes("node_nodecc")
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    b, res, texts = _run([data], "device")
    assert res[0]["status"] == 0
    _check_segments(b.segments(0))
    assert hashlib.sha256(texts[0]).hexdigest() == hashlib.sha256(want).hexdigest()


def test_segmenting_off_replays_whole(monkeypatch):
    monkeypatch.setenv("DTGPU_SEG", "0")
    data = G.dt_bytes("node_nodecc")
    b, res, texts = _run([data], "device")
    assert res[0]["status"] == 0 and b.segments(0) == []
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    assert texts[0] == want


def test_forced_segments_synthetic(monkeypatch):
    """Phased synthetic documents (concurrency up to every cut): the segmented texts equal
    the oracle's."""
    monkeypatch.setenv("DTGPU_SEG_OPS", "12")
    docs = [phased_doc(s) for s in range(6)]
    b, res, texts = _run(docs, "device")
    for i, d in enumerate(docs):
        assert res[i]["status"] == 0, (i, res[i])
        assert texts[i] == OracleOpLog.load_from(d).checkout_tip_bytes(), i
        _check_segments(b.segments(i), 3)


def test_forced_segments_debug_invariants(monkeypatch):
    """DTGPU_DEBUG=1 checks the whole index after every command: the placeholder blocks a
    segment starts from must be a consistent index."""
    monkeypatch.setenv("DTGPU_SEG_OPS", "400")
    monkeypatch.setenv("DTGPU_DEBUG", "1")
    b, res, texts = _run([G.dt_bytes("friendsforever")], "device")
    assert res[0]["status"] == 0, res[0]
    assert texts[0] == _ff_want()
    _check_segments(b.segments(0))


def test_forced_segments_lds_handback(monkeypatch):
    """An LDS index sized far too small: segments overflow it and replay again on the HBM
    tier, placeholders included."""
    monkeypatch.setenv("DTGPU_SEG_OPS", "300")
    monkeypatch.setenv("DTGPU_LDS_FILL", "4000")
    b, res, texts = _run([G.dt_bytes("friendsforever")] * 2, "device")
    assert [r["status"] for r in res] == [0, 0]
    assert all(t == _ff_want() for t in texts)
    _check_segments(b.segments(0), 4)


def _scattered_inserts_doc(seed, n_ins=400):
    """A concurrent prefix (two agents, then a merge: the history has cut points only after it),
    then long inserts (16-48 chars) scattered over the whole text and a few deletes: with small
    segments each later segment's inserts land across many placeholder blocks, the case the
    block reservation of add_segments (dtgpu_api.cpp) bounds."""
    import random
    rng = random.Random(seed)
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("a")
    b = o.get_or_create_agent_id("b")
    for k in range(60):
        o.add_insert(a, 0, "".join(rng.choice("abcdefgh") for _ in range(100)))
    v = o.local_frontier()
    x = o.add_insert_at(a, v, 10, "AAAA")
    y = o.add_insert_at(b, v, 20, "BBBB")
    o.add_insert_at(a, [x, y], 0, "merge")
    n = 6000 + 13
    for k in range(n_ins):
        if k % 10 == 9 and n > 100:
            p = rng.randrange(n - 30)
            o.add_delete_without_content(a if k % 20 else b, p, p + 20)
            n -= 20
        else:
            s = "".join(rng.choice("ijklmnop") for _ in range(rng.randint(16, 48)))
            o.add_insert(b if k % 3 else a, rng.randint(0, n), s)
            n += len(s)
    return o.encode()


def test_segments_with_scattered_long_inserts(monkeypatch):
    monkeypatch.setenv("DTGPU_SEG_OPS", "24")
    docs = [_scattered_inserts_doc(s) for s in range(3)]
    b, res, texts = _run(docs, "device")
    for i, d in enumerate(docs):
        assert res[i]["status"] == 0, (i, res[i])
        assert texts[i] == OracleOpLog.load_from(d).checkout_tip_bytes(), i
        _check_segments(b.segments(i), 4)


def _many_entries_doc(rounds):
    """2 * rounds + 1 graph entries: each round two agents insert at the same version, the next
    round merges them."""
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("a")
    b = o.get_or_create_agent_id("b")
    v = [o.add_insert(a, 0, "start")]
    n = 5
    for r in range(rounds):
        x = o.add_insert_at(a, v, r % n, "x")
        y = o.add_insert_at(b, v, (r * 7) % n, "y")
        v = [x, y]
        n += 2
    return o.encode()


def test_walk_kernel_past_64k_lds():
    """~16k graph entries (near PLAN_MAX_LDS_ENTRIES): the walk kernel's stack and pending counts
    take more than the default 64 KiB of dynamic LDS (dt_plan.hip launch_walk raises the
    limit); device-planned, text equal to the oracle's."""
    d = _many_entries_doc(8000)
    o = dt_amd.ListOpLog.load_from(d)
    assert 16000 <= len(o.export("entries")) <= 16384
    b, res, texts = _run([d], "device")
    assert res[0]["status"] == 0, res[0]
    assert b.host_planned() == [0]
    assert texts[0] == OracleOpLog.load_from(d).checkout_tip_bytes()
