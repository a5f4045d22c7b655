"""`OpLog::checkout_text` (src/oplog.rs:388-394) -> `TextInfo::merge_into`
(src/listmerge/merge.rs:954-1054): one text CRDT whose ops are some of the LV spans of a shared
causal graph is checked out over the graph projected onto those spans (`Graph::subgraph_raw` /
`project_onto_subgraph_raw`, src/causalgraph/graph/subgraph.rs:39-250).  libdtgpu builds the
projected sub-oplog on the host (dtgpu_oplog_project) and checks it out on the device.

The reference's multi-CRDT `OpLog` file format is not part of this path, so the shared graph is
built here: the ops of a text A (a benchmark file or a synthetic document) interleaved with the
ops of a second text B, where B ops relay A's dependencies (an A entry's parents become a chain
of B ops whose first member has the A parents) and other B ops hang off A ops.  The projection
onto A must then give back A's own causal order: the same ops keyed by (agent, seq) with the same
parents, so the oracle's checkout of the rebuilt projection equals its checkout of A.  Parity is
anchored on the oracle's checkout of A (itself pinned on the reference's golden vectors); the
multi-CRDT container itself is "parity unpinned" (no reference fixture holds one).  The projection
is pinned by the reference's own subgraph KATs (subgraph.rs:353-380 over fancy_graph, below).
"""
import random

import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog
from test_checkout_version import _oracle_rebuild
from test_encoder import _keyed
import dt_amd

RELAY = "~relay"


def _interleave(a, seed, p_relay=0.3, p_noise=0.2):
    """Shared graph of text A (the engine oplog `a`) and relay / noise text B.  Returns
    (combined oplog, A's LV spans in it, B's LV spans, number of B ops)."""
    rng = random.Random(seed)
    names = [n.decode() if isinstance(n, bytes) else n for n in a.export("agent_names")]
    c = dt_amd.ListOpLog()
    ids = [c.get_or_create_agent_id(n) for n in names]
    relay = c.get_or_create_agent_id(RELAY)
    ents = a.export("entries").reshape(-1, 2)
    off = a.export("parent_offsets")
    par = a.export("parents")
    starts = {int(s): [int(x) for x in par[off[i]:off[i + 1]]] for i, (s, _e) in enumerate(ents)}
    content = bytes(a.export("content"))
    coff = a.export("char_offsets")
    agent_of = {}
    for lv, ln, agent, _seq in a.export("agent_runs").reshape(-1, 4):
        for k in range(int(ln)):
            agent_of[int(lv) + k] = ids[int(agent)]
    amap = {}          # A LV -> combined LV
    a_lvs, b_lvs = [], []
    n_b = 0

    def add_b(parents):
        nonlocal n_b
        v = c.add_insert_at(relay, parents, 0, "x")
        b_lvs.append(v)
        n_b += 1
        return v

    for lv, ln, pos, kf in a.export("ops").reshape(-1, 4):
        lv, ln, pos, kind, fwd = int(lv), int(ln), int(pos), int(kf) & 1, (int(kf) >> 1) & 1
        for k in range(ln):
            v = lv + k
            ps = [amap[p] for p in starts.get(v, [v - 1] if v else [])]
            if v in starts and rng.random() < p_relay:
                for _ in range(rng.choice([1, 1, 2])):
                    ps = [add_b(ps)]
            if kind == 0:
                b = int(coff[v])
                ch = content[b:b + 4].decode("utf-8", errors="ignore")[:1]
                nv = c.add_insert_at(agent_of[v], ps, pos + k, ch)
            else:
                p = pos if fwd else pos + ln - 1 - k
                nv = c.add_delete_at(agent_of[v], ps, p, p + 1)
            amap[v] = nv
            a_lvs.append(nv)
            if rng.random() < p_noise:
                add_b([nv])
    return c, _spans(a_lvs), _spans(b_lvs), n_b


def _spans(lvs):
    out = []
    for v in sorted(lvs):
        if out and out[-1][1] == v:
            out[-1][1] = v + 1
        else:
            out.append([v, v + 1])
    return [tuple(x) for x in out]


def _a_docs():
    yield "friendsforever", dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever")), \
        OracleOpLog.load_from(G.dt_bytes("friendsforever")).checkout_tip_bytes()
    for doc in (0, 5):
        o = dt_amd.synth_oplog(doc, 1500)
        yield f"synth{doc}", o, _oracle_rebuild(o).checkout_tip_bytes()


@pytest.mark.parametrize("seed", [1, 2])
def test_projection_gives_back_the_text_order(seed):
    for name, a, want in _a_docs():
        c, a_spans, b_spans, n_b = _interleave(a, seed)
        assert n_b > 0 and len(a_spans) > 1
        sub = c.project(a_spans)
        assert len(sub) == len(a)
        assert _keyed(sub) == _keyed(a), name
        assert _oracle_rebuild(sub).checkout_tip_bytes() == want, name
        # the projected version is A's frontier (as (agent, seq) ids)
        key = {}
        for lv, ln, agent, seq in sub.export("agent_runs").reshape(-1, 4):
            for k in range(int(ln)):
                key[int(lv) + k] = (int(agent), int(seq) + k)
        akey = {}
        for lv, ln, agent, seq in a.export("agent_runs").reshape(-1, 4):
            for k in range(int(ln)):
                akey[int(lv) + k] = (int(agent), int(seq) + k)
        assert sorted(key[v] for v in sub.local_frontier()) == sorted(akey[v] for v in a.local_frontier())


def test_projection_of_the_relay_text():
    """B's ops hang off A's, so B's projected versions are wide antichains (thousands wide on
    friendsforever); every B op inserts "x" at 0, so its text is n_B x's."""
    for a in (dt_amd.synth_oplog(2, 1500), dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))):
        c, _a_spans, b_spans, n_b = _interleave(a, 3)
        sub = c.project(b_spans)
        assert len(sub) == n_b
        assert _oracle_rebuild(sub).checkout_tip_bytes() == b"x" * n_b


def test_projection_onto_everything_and_onto_a_history():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    full = o.project([(0, len(o))])
    assert _keyed(full) == _keyed(o) and full.local_frontier() == o.local_frontier()
    rng = random.Random(4)
    for _ in range(3):
        v = o.dominators([rng.randrange(len(o))])
        h = o.history(v)
        hist = [tuple(x) for x in _hist_spans(o, v)]
        sub = o.project(hist)
        assert _keyed(sub) == _keyed(h)


def _hist_spans(o, v):
    """Hist(v) as ascending spans, from the projection-free history sub-oplog's size and the
    graph: every LV whose entry is reachable from v (brute force over the exported parents)."""
    ents = o.export("entries").reshape(-1, 2)
    off = o.export("parent_offsets")
    par = o.export("parents")
    starts = np.asarray(ents[:, 0])

    def entry_of(x):
        return int(np.searchsorted(starts, x, side="right") - 1)

    top = {}   # entry -> highest LV of it in the history
    stack = list(v)
    while stack:
        x = stack.pop()
        e = entry_of(x)
        if top.get(e, -1) >= x:
            continue
        top[e] = x
        stack.extend(int(p) for p in par[off[e]:off[e + 1]])
    return _spans([lv for e, x in top.items() for lv in range(int(ents[e][0]), x + 1)])


def test_projection_rejects_bad_spans():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    with pytest.raises(dt_amd.ParseError):
        o.project([(0, len(o) + 1)])
    assert len(o.project([])) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1])
def test_gpu_checkout_text(seed):
    for name, a, want in _a_docs():
        c, a_spans, b_spans, n_b = _interleave(a, seed)
        assert c.checkout_text_bytes(a_spans) == want, name
        assert c.checkout_text_bytes(b_spans) == b"x" * n_b, name


# ---- Graph::subgraph KATs (src/causalgraph/graph/subgraph.rs:353-380, test_subgraph) -------------
# fancy_graph (graph/tools.rs:903-919): 0..3 and 3..6 from ROOT, 6..9 after [1, 4], 9..11 after
# [2, 8].  check_subgraph(filter, frontier, parents of each subgraph entry, projected frontier);
# the reference keeps LV numbering, libdtgpu compacts it (history at `frontier`, then the
# projection), so the expectations are mapped through both compactions.
FANCY = [(0, 3, []), (3, 6, []), (6, 9, [1, 4]), (9, 11, [2, 8])]
SUBGRAPH_KATS = [
    ([(0, 11)], [5, 10], [[], [], [1, 4], [2, 8]], [5, 10]),
    ([(1, 11)], [5, 10], [[], [], [1, 4], [2, 8]], [5, 10]),
    ([(5, 6)], [5, 10], [[]], [5]),
    ([(0, 1), (10, 11)], [5, 10], [[], [0]], [10]),
    ([(0, 11)], [10], [[], [], [1, 4], [2, 8]], [10]),
    ([(0, 11)], [5], [[]], [5]),
    ([(0, 3), (9, 11)], [10], [[], [2]], [10]),
    ([(9, 11)], [3], [], []),
    ([(5, 6)], [9], [], []),
    ([(0, 1), (2, 3)], [2], [[], [0]], [2]),
    ([(0, 1), (2, 3)], [9], [[], [0]], [2]),
]


def _fancy_oplog():
    o = dt_amd.ListOpLog()
    for i, (s, e, par) in enumerate(FANCY):
        a = o.get_or_create_agent_id("abcd"[i])
        assert o.add_insert_at(a, par, 0, "xyz"[:e - s]) == e - 1
    return o


def _hist(frontier):
    ents = {v: (s, par) for s, e, par in FANCY for v in range(s, e)}
    seen, todo = set(), list(frontier)
    while todo:
        v = todo.pop()
        if v in seen:
            continue
        seen.add(v)
        s, par = ents[v]
        todo += par if v == s else [v - 1]
    return sorted(seen)


@pytest.mark.parametrize("kat", range(len(SUBGRAPH_KATS)))
def test_projection_matches_reference_subgraph_kats(kat):
    filt, frontier, expect_parents, expect_frontier = SUBGRAPH_KATS[kat]
    hist = _hist(frontier)
    h_of = {v: i for i, v in enumerate(hist)}                       # original -> history LV
    inside = [v for v in hist if any(a <= v < b for a, b in filt)]
    t_of = {v: i for i, v in enumerate(inside)}                     # original -> projected LV
    h = _fancy_oplog().history(frontier)
    sub = h.project(_spans(h_of[v] for v in inside))
    assert len(sub) == len(inside)
    # per-LV parents (an entry's first LV: its parents; the others: the previous LV), so RLE
    # merging of adjacent entries does not matter
    ents = sub.export("entries").reshape(-1, 2)
    off = sub.export("parent_offsets")
    par = sub.export("parents")
    got = {}
    for i, (a, b) in enumerate(ents):
        for v in range(int(a), int(b)):
            got[v] = sorted(int(x) for x in par[off[i]:off[i + 1]]) if v == a else [v - 1]
    # the reference's subgraph entries: runs of diff(frontier) n filter split at its txns
    starts = {s0 for s0, _e, _p in FANCY}
    runs = []
    for v in inside:
        if runs and runs[-1][-1] == v - 1 and v not in starts:
            runs[-1].append(v)
        else:
            runs.append([v])
    assert len(runs) == len(expect_parents)
    want = {}
    for run, ps in zip(runs, expect_parents):
        for v in run:
            want[t_of[v]] = sorted(t_of[p] for p in ps) if v == run[0] else [t_of[v] - 1]
    assert got == want, (kat, got, want)
    assert sorted(int(x) for x in sub.local_frontier()) == sorted(t_of[v] for v in expect_frontier)


@pytest.mark.parametrize("kat", range(len(SUBGRAPH_KATS)))
def test_project_version_matches_reference_subgraph_kats(kat):
    """Graph::project_onto_subgraph_raw as the reference's KATs state it (subgraph.rs:353-380):
    the projection of `frontier` onto the filter, over fancy_graph itself (dtgpu_oplog_project_version;
    projected LVs are the filter's LVs in ascending order)."""
    filt, frontier, _parents, expect_frontier = SUBGRAPH_KATS[kat]
    members = [v for a, b in sorted(filt) for v in range(a, b)]
    idx = {v: i for i, v in enumerate(members)}
    assert _fancy_oplog().project_version(filt, frontier) == sorted(idx[v] for v in expect_frontier)


def test_project_version_of_the_tip_is_the_sub_oplog_frontier():
    a = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    c, a_spans, b_spans, _n = _interleave(a, 3)
    for spans in (a_spans, b_spans):
        assert c.project_version(spans, c.local_frontier()) == c.project(spans).local_frontier()
        assert c.project_version(spans, []) == []
