"""`ListOpLog::checkout(&[LV])` (src/list/oplog.rs:32-36), `Graph::find_dominators_2`
(src/causalgraph/graph/tools.rs:545-578) and `ListBranch::merge` from a non-ROOT version
(src/list/merge.rs:63-95).

CPU tests pin the host side: the frontier of a union of versions against brute-force
reachability in the oracle's graph (`dto_graph_contains`), and the history sub-oplog that the
device checks out (`dtgpu_oplog_history`) rebuilt in the oracle, whose tip checkout must equal
the oracle's own walk of Hist(version).  GPU tests compare the device checkout at a version and
branch merges with the oracle byte for byte.
"""
import random

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, lib as oracle_lib
import dt_amd


def _graph_of(o):
    """The oracle's Graph built from the engine's exported entries."""
    import ctypes
    ents = o.export("entries").reshape(-1, 2)
    off = o.export("parent_offsets")
    par = o.export("parents")
    L = oracle_lib()
    g = L.dto_graph_new()
    for i, (s, e) in enumerate(ents):
        ps = [int(x) for x in par[off[i]:off[i + 1]]]
        a = (ctypes.c_int64 * max(1, len(ps)))(*ps)
        L.dto_graph_push(g, a, len(ps), int(s), int(e))
    return g


def _contains(g, frontier, v):
    import ctypes
    a = (ctypes.c_int64 * max(1, len(frontier)))(*frontier)
    return bool(oracle_lib().dto_graph_contains(g, a, len(frontier), v))


def _versions(n_lv, rng, k=12):
    out = [[], [n_lv - 1]]
    for _ in range(k):
        m = rng.choice([1, 1, 2, 3])
        out.append(sorted(rng.sample(range(n_lv), m)))
    return out


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_dominators_match_reachability(name):
    o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
    g = _graph_of(o)
    rng = random.Random(7)
    try:
        vs = _versions(len(o), rng, 20)
        for a in vs:
            for b in rng.sample(vs, 4):
                got = o.dominators(a, b)
                u = sorted(set(a) | set(b))
                want = [v for v in u if not any(w != v and _contains(g, [w], v) for w in u)]
                assert got == want, (a, b)
    finally:
        oracle_lib().dto_graph_free(g)
    with pytest.raises(ValueError):
        o.dominators([len(o)])


def _oracle_rebuild(sub):
    """Rebuild an engine oplog in the oracle one LV at a time (same agents, parents, positions)."""
    names = sub.export("agent_names")
    ora = OracleOpLog()
    ids = [ora.agent(n.decode() if isinstance(n, bytes) else n) for n in names]
    ents = sub.export("entries").reshape(-1, 2)
    off = sub.export("parent_offsets")
    par = sub.export("parents")
    content = bytes(sub.export("content"))
    coff = sub.export("char_offsets")
    agent_of = {}
    for lv, ln, agent, _seq in sub.export("agent_runs").reshape(-1, 4):
        for k in range(int(ln)):
            agent_of[int(lv) + k] = ids[int(agent)]
    parents_of = {}
    for i, (s, e) in enumerate(ents):
        parents_of[int(s)] = [int(x) for x in par[off[i]:off[i + 1]]]
    for lv, ln, pos, kf in sub.export("ops").reshape(-1, 4):
        lv, ln, pos, kind, fwd = int(lv), int(ln), int(pos), int(kf) & 1, (int(kf) >> 1) & 1
        for k in range(ln):
            v = lv + k
            ps = parents_of.get(v, [v - 1])
            if kind == 0:
                b = int(coff[v])
                ch = content[b:b + 4].decode("utf-8", errors="ignore")[:1]
                ora.add_insert_at(agent_of[v], ps, pos + k, ch)
            else:
                p = pos if fwd else pos + ln - 1 - k
                ora.add_delete_at(agent_of[v], ps, p, p + 1)
    return ora


@pytest.mark.parametrize("name", ["friendsforever"])
def test_history_suboplog_is_the_checkout_at_version(name):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    ora = OracleOpLog.load_from(data)
    rng = random.Random(11)
    for v in _versions(len(o), rng, 6):
        v = o.dominators(v)
        sub = o.history(v)
        want = ora.checkout_bytes(v)
        rebuilt = _oracle_rebuild(sub)
        assert len(rebuilt) == len(sub)
        assert rebuilt.checkout_tip_bytes() == want, v


def test_history_of_synthetic_docs():
    rng = random.Random(3)
    for doc in range(3):
        o = dt_amd.synth_oplog(doc, 1500)
        ora = _oracle_rebuild(o)
        for v in _versions(len(o), rng, 4):
            v = o.dominators(v)
            assert _oracle_rebuild(o.history(v)).checkout_tip_bytes() == ora.checkout_bytes(v), (doc, v)


def test_history_root_and_tip():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    assert len(o.history([])) == 0
    tip = o.history(o.local_frontier())
    assert len(tip) == len(o)
    assert tip.local_frontier() == o.local_frontier()


# ---- GPU ----------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_gpu_checkout_at_version_matches_oracle(name):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    ora = OracleOpLog.load_from(data)
    rng = random.Random(5)
    for v in _versions(len(o), rng, 8 if name == "friendsforever" else 3):
        br = o.checkout(v)
        assert br.local_frontier() == o.dominators(v)
        assert br.content_bytes() == ora.checkout_bytes(br.local_frontier()), v


@pytest.mark.gpu
def test_gpu_checkout_root_is_empty():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    br = o.checkout([])
    assert br.content() == "" and br.local_frontier() == []


@pytest.mark.gpu
def test_gpu_branch_merge_from_non_root():
    data = G.dt_bytes("friendsforever")
    o = dt_amd.ListOpLog.load_from(data)
    ora = OracleOpLog.load_from(data)
    rng = random.Random(9)
    br = dt_amd.ListBranch.new()
    for _ in range(6):
        f = [rng.randrange(len(o))]
        br.merge(o, f)
        assert br.content_bytes() == ora.checkout_bytes(br.local_frontier())
    br.merge(o, o.local_frontier())
    assert br.content() == G.trace("friendsforever_flat")["endContent"]
    assert br.local_frontier() == o.local_frontier()


@pytest.mark.gpu
def test_gpu_checkout_at_version_synthetic():
    rng = random.Random(13)
    for doc in range(4):
        o = dt_amd.synth_oplog(doc, 2000)
        ora = _oracle_rebuild(o)
        for v in _versions(len(o), rng, 3):
            br = o.checkout(v)
            assert br.content_bytes() == ora.checkout_bytes(br.local_frontier()), (doc, v)
