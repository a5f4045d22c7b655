"""Cut points of a causal graph (dtgpu_oplog_cut_ranges), the foundation of the cut replay
(dt_replay.hip "segments"): an LV v is a cut when the ops below v form the single version {v-1}
and every later op has v-1 in its history -- the state the reference fast-forwards across
(src/listmerge/merge.rs:811-840).  The linear-time computation is checked against the
definition evaluated by brute force (per-LV history bitsets) on synthetic histories, and
pinned on the benchmark files."""
import pytest

import golden_data as G
from synth_docs import phased_doc

import dt_amd


def _brute_cuts(o):
    """Maximal ranges of cuts straight from the definition (small documents only)."""
    ent = o.export("entries")
    po, par = o.export("parent_offsets"), o.export("parents")
    n = len(o)
    parents = [None] * n
    for k, (s, e) in enumerate(ent):
        for x in range(int(s), int(e)):
            parents[x] = [int(p) for p in par[po[k]:po[k + 1]]] if x == s else [x - 1]
    hist = [0] * n   # bitset of each LV's history (itself included)
    minchild = [n + 1] * n
    for x in range(n):
        h = 1 << x
        for p in parents[x]:
            h |= hist[p]
            minchild[p] = min(minchild[p], x)
        hist[x] = h
    cuts = []
    for v in range(1, n + 1):
        # frontier of [0, v) is {v-1}: every y < v-1 has a child below v
        if any(minchild[y] >= v for y in range(v - 1)):
            continue
        if all((hist[x] >> (v - 1)) & 1 for x in range(v, n)):
            cuts.append(v)
    ranges = []
    for v in cuts:
        if ranges and ranges[-1][1] == v - 1:
            ranges[-1][1] = v
        else:
            ranges.append([v, v])
    return [tuple(r) for r in ranges]


def _merged(ranges):
    out = []
    for a, b in ranges:
        if out and out[-1][1] + 1 >= a:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [tuple(r) for r in out]


@pytest.mark.parametrize("seed", range(5))
def test_cut_ranges_match_definition(seed):
    o = dt_amd.ListOpLog.load_from(phased_doc(seed, phases=6))
    assert len(o) < 1500
    got = _merged(o.cut_ranges())
    assert got == _brute_cuts(o)
    assert len(got) >= 3


def test_cut_ranges_linear_and_concurrent_edges():
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("a")
    o.add_insert(a, 0, "hello")
    o.add_insert(a, 5, " world")
    assert _merged(o.cut_ranges()) == [(1, len(o))] == _brute_cuts(o)
    # two concurrent roots and no merge: nothing is ever one version seen by everything after
    c = dt_amd.ListOpLog()
    x, y = c.get_or_create_agent_id("x"), c.get_or_create_agent_id("y")
    c.add_insert_at(x, [], 0, "ab")
    c.add_insert_at(y, [], 0, "cd")
    assert _merged(c.cut_ranges()) == _brute_cuts(c)


def test_cut_ranges_benchmark_files():
    """node_nodecc: eight ranges, the last one its whole second half; git-makefile: only its
    last few LVs (every branch forks from an older version)."""
    node = dt_amd.ListOpLog.load_from(G.dt_bytes("node_nodecc"))
    r = node.cut_ranges()
    assert len(r) == 8 and r[0] == (1, 63277) and r[-1] == (450964, len(node))
    git = dt_amd.ListOpLog.load_from(G.dt_bytes("git-makefile"))
    assert git.cut_ranges() == [(348793, len(git))]
    ff = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    assert len(ff.cut_ranges()) == 147
