"""GPU parity: libdtgpu's device checkout vs the CPU oracle and the reference's golden texts.

Every test calls through the C ABI (dt_amd -> libdtgpu.so -> HIP kernels).  Bit-exact bar:
the merged text must equal the oracle's / golden bytes exactly.
"""
import hashlib

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, oplog_from_trace as oracle_from_trace

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def test_friendsforever_golden():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    assert len(o) == 26078
    br = o.checkout_tip()
    assert br.content() == G.trace("friendsforever_flat")["endContent"]
    assert br.local_frontier() == [26077]


@pytest.mark.parametrize("vec", [G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_LZ4])
def test_compat_simple(vec):
    assert dt_amd.ListOpLog.load_from(vec).checkout_tip().content() == "hi me"


@pytest.mark.parametrize("vec", [G.COMPAT_EMPTY_1, G.COMPAT_EMPTY_2])
def test_compat_empty(vec):
    assert dt_amd.ListOpLog.load_from(vec).checkout_tip().content() == ""


@pytest.mark.parametrize("name", ["git-makefile", "node_nodecc"])
def test_large_docs_vs_oracle(name):
    data = G.dt_bytes(name)
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    got = dt_amd.ListOpLog.load_from(data).checkout_tip_bytes()
    assert len(got) == len(want)
    assert hashlib.sha256(got).hexdigest() == hashlib.sha256(want).hexdigest()


@pytest.mark.parametrize("name", G.JSON_TRACES)
def test_json_traces_golden(name):
    t = G.trace(name)
    o = dt_amd.oplog_from_trace(t["txns"])
    assert o.checkout_tip().content() == t["endContent"]


def test_batch_friendsforever_copies():
    data = G.dt_bytes("friendsforever")
    want = G.trace("friendsforever_flat")["endContent"].encode()
    b = dt_amd.Batch(docs=[bytes(data) for _ in range(300)])
    b.run()
    b.sync()
    res = b.results()
    h = dt_amd.text_hash(want)
    assert all(r["status"] == 0 and r["text_len"] == len(want) and r["text_hash"] == h for r in res)
    assert b.text(0) == want and b.text(299) == want


def test_batch_mixed_and_errors():
    docs = [G.dt_bytes("friendsforever"), b"not a dt file", G.COMPAT_SIMPLE_LZ4, G.dt_bytes("git-makefile"),
            G.COMPAT_EMPTY_2]
    bad = bytearray(G.COMPAT_SIMPLE_1)
    bad[-1] ^= 0xFF
    docs.append(bytes(bad))
    res, texts = dt_amd.batch_checkout(docs)
    assert [r["status"] for r in res] == [0, 1, 0, 0, 0, 18]
    assert texts[0].decode() == G.trace("friendsforever_flat")["endContent"]
    assert texts[2] == b"hi me" and texts[4] == b""
    assert texts[3] == OracleOpLog.load_from(G.dt_bytes("git-makefile")).checkout_tip_bytes()


def _kat(build):
    g = dt_amd.ListOpLog()
    o = OracleOpLog()
    build(g, o)
    return g.checkout_tip().content(), o.checkout_tip()


def test_merge_kats():
    def b1(g, o):
        for x in (g, o):
            ag = x.get_or_create_agent_id if x is g else x.agent
            a, b = ag("a"), ag("b")
            x.add_insert_at(a, [], 0, "aaa")
            x.add_insert_at(b, [], 0, "bbb")
            x.add_insert_at(a, [2, 5], 0, "ccc")
    got, want = _kat(b1)
    assert got == want == "cccaaabbb"

    def b2(g, o):
        for x in (g, o):
            ag = x.get_or_create_agent_id if x is g else x.agent
            a, b = ag("a"), ag("b")
            t = x.add_insert_at(a, [], 0, "aaa")
            x.add_delete_at(a, [t], 1, 2)
            x.add_delete_at(b, [t], 0, 3)
    got, want = _kat(b2)
    assert got == want == ""


def test_unicode():
    g = dt_amd.ListOpLog()
    s = g.get_or_create_agent_id("seph")
    g.add_insert(s, 0, "héllo 𝄞 wörld")
    g.add_delete_without_content(s, 1, 2)
    g.add_insert(s, 6, "✓")
    assert g.checkout_tip().content() == "hllo 𝄞✓ wörld"


def _with_env(env, fn):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_lds_overflow_falls_back_to_hbm_tier():
    """An optimistic LDS capacity far too small: every document overflows in the LDS tier and is
    replayed by the HBM tier inside the same run; texts must still be exact."""
    data = G.dt_bytes("friendsforever")
    want = G.trace("friendsforever_flat")["endContent"].encode()

    def run():
        b = dt_amd.Batch(docs=[data] * 70 + [G.COMPAT_SIMPLE_LZ4])
        b.run()
        b.sync()
        return b.results(), b.text(0), b.text(69), b.text(70)

    res, t0, t69, t70 = _with_env({"DTGPU_LDS_FILL": "400"}, run)
    assert all(r["status"] == 0 for r in res)
    assert t0 == want and t69 == want and t70 == b"hi me"


def test_invariants_hold_after_every_command():
    """DTGPU_DEBUG=1 checks the whole tree (masks vs per-item counts, block / superblock totals,
    positions) after every command of the replay."""
    for name in ("friendsforever",):
        data = G.dt_bytes(name)
        got = _with_env({"DTGPU_DEBUG": "1"}, lambda: dt_amd.ListOpLog.load_from(data).checkout_tip_bytes())
        assert got == G.trace("friendsforever_flat")["endContent"].encode()
    g = _with_env({"DTGPU_DEBUG": "1"}, lambda: dt_amd.ListOpLog.load_from(G.COMPAT_SIMPLE_LZ4).checkout_tip_bytes())
    assert g == b"hi me"


def _host_plan(oplog):
    return oplog.plan_commands(), oplog.plan_tlist()


def _same_plan(gpu, host):
    """Same command sequence; a TOG's entries compared as a multiset (the pass is commutative)."""
    (gc, gt), (hc, ht) = gpu, host
    assert len(gc) == len(hc)
    for k, (a, b) in enumerate(zip(gc, hc)):
        assert a[0] == b[0], (k, a, b)
        if (a[0] & 15) == 2:
            assert a[2] == b[2], (k, a, b)
            assert sorted(gt[a[1]:a[1] + a[2]]) == sorted(ht[b[1]:b[1] + b[2]]), k
        else:
            assert a == b, (k, a, b)


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile", "node_nodecc"])
def test_device_planner_matches_host_walk(name):
    """dt_plan.hip walks the graph in the reference's spanning-tree order and derives the
    retreat / advance sets from agent version vectors: its stream must equal the host planner's
    (Graph::diff_rev) command for command."""
    data = G.dt_bytes(name)
    b = dt_amd.Batch(docs=[data])
    assert b.host_planned() == [0]
    b.run()
    b.sync()
    _same_plan(b.plan(0), _host_plan(dt_amd.ListOpLog.load_from(data)))


def test_device_planner_on_traces_and_kats():
    oplogs = [dt_amd.oplog_from_trace(G.trace(n)["txns"]) for n in ("sveltecomponent", "friendsforever_flat")]
    g = dt_amd.ListOpLog()
    a, c = g.get_or_create_agent_id("a"), g.get_or_create_agent_id("b")
    t = g.add_insert_at(a, [], 0, "aaa")
    g.add_insert_at(c, [], 0, "bbb")
    g.add_delete_at(c, [t], 0, 2)
    g.add_insert_at(a, [2, 5], 0, "ccc")
    oplogs.append(g)
    # the linear traces check out on the fast-forward path by default (dt_ff.hip, no walk plan);
    # the planner is compared on them with that path off
    assert dt_amd.Batch(oplogs=oplogs).fast_forwarded() == [1, 1, 0]
    b = _with_env({"DTGPU_FF": "0"}, lambda: dt_amd.Batch(oplogs=oplogs))
    assert b.host_planned() == [0] * 3
    b.run()
    b.sync()
    for i, o in enumerate(oplogs):
        _same_plan(b.plan(i), _host_plan(o))
    assert b.text(2) == OracleOpLog_from(g).encode()


def OracleOpLog_from(g):
    """Rebuild the KAT oplog in the oracle and check it out there."""
    o = OracleOpLog()
    a, c = o.agent("a"), o.agent("b")
    t = o.add_insert_at(a, [], 0, "aaa")
    o.add_insert_at(c, [], 0, "bbb")
    o.add_delete_at(c, [t], 0, 2)
    o.add_insert_at(a, [2, 5], 0, "ccc")
    return o.checkout_tip()


def test_host_planner_path_still_exact():
    data = G.dt_bytes("git-makefile")
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    b = _with_env({"DTGPU_HOST_PLAN": "1"}, lambda: dt_amd.Batch(docs=[data, G.dt_bytes("friendsforever")]))
    assert b.host_planned() == [1, 1]
    b.run()
    b.sync()
    assert b.text(0) == want


def test_synthetic_docs_vs_oracle():
    """Synthetic concurrent docs (4-16 agents, epochs of concurrent edits): device checkout ==
    CPU oracle, and the device plan == the host plan."""
    from test_synth import oracle_from_synth
    docs = list(range(12))
    oplogs = [dt_amd.synth_oplog(d, 5000) for d in docs]
    b = dt_amd.Batch(oplogs=oplogs)
    assert b.host_planned() == [0] * len(docs)
    b.run()
    b.sync()
    for i, d in enumerate(docs):
        _, _, o = oracle_from_synth(d, 5000)
        assert b.text(i) == o.checkout_tip_bytes(), d
        _same_plan(b.plan(i), _host_plan(oplogs[i]))
