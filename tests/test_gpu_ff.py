"""The fast-forward checkout on the device (dt_ff.hip; merge.rs:811-840): linear histories --
the five JSON benchmark traces, random linear documents with multi-byte text, segment-boundary
sizes -- checked against the reference's endContent and the oracle, alone, in batches, beside
tracker documents (configs[4]'s mix), through the timed pass and the e2e pass, and against the
per-item tracker on the same documents (DTGPU_FF=0)."""
import os

import pytest

import golden_data as G
import linear_docs as L
from oracle.oracle import OpLog as OracleOpLog

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module")
def traces():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")
    out = []
    for n in G.JSON_TRACES:
        t = G.trace(n)
        out.append((n, dt_amd.apply_edits_push_merge(t["txns"]).encode(), t["endContent"].encode()))
    return out


def check(b, want):
    res = b.results()
    for i, (r, w) in enumerate(zip(res, want)):
        assert r["status"] == 0, (i, r)
        assert (r["text_len"], r["text_hash"]) == (len(w), dt_amd.text_hash(w)), i
        assert b.text(i) == w, i


def test_linear_traces_fast_forward_alone(traces):
    for name, data, want in traces:
        b = dt_amd.Batch(docs=[data], staging="device")
        assert b.fast_forwarded() == [1], name
        b.run()
        b.sync()
        check(b, [want])
        b.run_timed()   # the timed pass rewrites the same text
        check(b, [want])
        assert b.segments(0) == []


def test_linear_traces_batch_and_e2e(traces):
    docs, want = [], []
    for k in range(3):
        for _, d, w in traces:
            docs.append(d)
            want.append(w)
    b = dt_amd.Batch(docs=docs, staging="device")
    assert b.fast_forwarded() == [1] * len(docs)
    b.run()
    b.sync()
    check(b, want)
    b.run_e2e_timed()   # decode -> fast-forward from the .dt bytes in HBM
    check(b, want)


def test_fast_forward_beside_tracker_documents(traces):
    """configs[4]'s mix: the three .dt files replay on the tracker, the linear traces fast-forward,
    in one pass (the split pass when critical documents exist)."""
    docs, want, ff = [], [], []
    for n in G.DT_FILES:
        d = G.dt_bytes(n)
        docs.append(d)
        want.append(OracleOpLog.load_from(d).checkout_tip_bytes())
        ff.append(0)
    for _, d, w in traces:
        docs += [d, d]
        want += [w, w]
        ff += [1, 1]
    b = dt_amd.Batch(docs=docs, staging="device")
    assert b.fast_forwarded() == ff
    b.run()
    b.sync()
    check(b, want)
    b.run_timed()
    check(b, want)


@pytest.mark.parametrize("seed", range(6))
def test_random_linear_documents(seed):
    docs, want = [], []
    for k in range(8):
        d, w = L.random_linear(100 * seed + k, 200 + 400 * k, paste_p=0.05 if k % 2 else 0.0)
        assert OracleOpLog.load_from(d).checkout_tip_bytes() == w
        docs.append(d)
        want.append(w)
    b = dt_amd.Batch(docs=docs, staging="device")
    assert b.fast_forwarded() == [1] * len(docs)
    b.run()
    b.sync()
    check(b, want)


def test_segment_boundaries():
    docs, want = [], []
    for runs in [1, 2, 62, 63, 64, 126, 127, 128, 189, 190, 4000, 20000]:
        d, w = L.sized_linear(runs, seed=runs)
        docs.append(d)
        want.append(w)
    b = dt_amd.Batch(docs=docs, staging="device")
    assert b.fast_forwarded() == [1] * len(docs)
    b.run()
    b.sync()
    check(b, want)


def test_fast_forward_equals_tracker(traces):
    """The same linear documents through the per-item tracker (DTGPU_FF=0 at staging): same texts."""
    docs = [d for _, d, _ in traces] + [L.random_linear(7, 3000)[0]]
    os.environ["DTGPU_FF"] = "0"
    try:
        bt = dt_amd.Batch(docs=docs, staging="device")
    finally:
        del os.environ["DTGPU_FF"]
    assert bt.fast_forwarded() == [0] * len(docs)
    bt.run()
    bt.sync()
    bf = dt_amd.Batch(docs=docs, staging="device")
    bf.run()
    bf.sync()
    rt, rf = bt.results(), bf.results()
    for i in range(len(docs)):
        assert rt[i]["status"] == 0 and rf[i]["status"] == 0
        assert (rt[i]["text_len"], rt[i]["text_hash"]) == (rf[i]["text_len"], rf[i]["text_hash"])
        assert bt.text(i) == bf.text(i)


def test_empty_text_and_full_delete():
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("x")
    o.add_insert(a, 0, "hello world")
    o.add_delete_without_content(a, 0, 11)
    gone = o.encode()
    o2 = dt_amd.ListOpLog()
    a2 = o2.get_or_create_agent_id("y")
    o2.add_insert(a2, 0, "abc")
    one = o2.encode()
    b = dt_amd.Batch(docs=[gone, one, gone], staging="device")
    assert b.fast_forwarded() == [1, 1, 1]
    b.run()
    b.sync()
    check(b, [b"", b"abc", b""])


def test_encode_after_fast_forward(traces):
    """The batched encoder still sees every document's walk (staging plans the fast-forwarded
    documents too): device bytes equal the host encoder's."""
    docs = [d for _, d, _ in traces]
    b = dt_amd.Batch(docs=docs, staging="device")
    b.run()
    b.sync()
    b.encode()
    for i, d in enumerate(docs):
        assert b.encoded(i) == dt_amd.ListOpLog.load_from(d).encode(), i


def test_host_staged_and_checkout_tip(traces):
    """Host-staged batches and ListOpLog.checkout_tip() take the same path for linear histories."""
    docs = [d for _, d, _ in traces]
    want = [w for _, _, w in traces]
    b = dt_amd.Batch(docs=docs, staging="host")
    assert b.fast_forwarded() == [1] * len(docs)
    b.run()
    b.sync()
    check(b, want)
    for d, w in zip(docs, want):
        assert dt_amd.ListOpLog.load_from(d).checkout_tip_bytes() == w


def test_batch_opts_select_the_path(traces):
    """dtgpu_batch_opts carries the knobs (DTGPU_OPT_*): the same as the environment overrides."""
    docs = [d for _, d, _ in traces]
    want = [w for _, _, w in traces]
    b = dt_amd.Batch(docs=docs, staging="device", flags=dt_amd.OPT_NO_FAST_FORWARD)
    assert b.fast_forwarded() == [0] * len(docs)
    b.run()
    b.sync()
    check(b, want)
    b = dt_amd.Batch(docs=docs, staging="device", flags=dt_amd.OPT_NO_FAST_FORWARD | dt_amd.OPT_NO_SEGMENTS)
    b.run()
    b.sync()
    check(b, want)
    assert all(b.segments(i) == [] for i in range(len(docs)))
