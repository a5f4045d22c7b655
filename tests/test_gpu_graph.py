"""GPU causal-graph queries (dt_graph.hip) vs the reference's fixtures and the C oracle.

diff / find_conflicting / version_contains over every test_data/causal_graph fixture in one
batch (tools.rs:779-901 semantics), then random queries over the benchmark files' graphs
against the oracle's restatement (oracle/dt_oracle.c, pinned by the same fixtures).
"""
import random

import pytest

import golden_data as G
from oracle.oracle import Graph as OracleGraph

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _ranges(rs):
    return [tuple(r) for r in rs]


def test_fixtures_one_batch():
    graphs, queries, checks = [], [], []
    for case in G.cg_fixture("diff"):
        graphs.append(case["hist"])
        queries.append(("diff", len(graphs) - 1, case["a"], case["b"]))
        checks.append(case)
    for case in G.cg_fixture("conflicting"):
        graphs.append(case["hist"])
        queries.append(("conflict", len(graphs) - 1, case["a"], case["b"]))
        checks.append(case)
    for case in G.cg_fixture("version_contains"):
        graphs.append(case["hist"])
        queries.append(("contains", len(graphs) - 1, case["frontier"], case["target"]))
        checks.append(case)
    got = dt_amd.graph_queries(graphs, queries)
    for (kind, _g, _a, _b), case, ans in zip(queries, checks, got):
        if kind == "diff":
            assert ans == (_ranges(case["expect_a"]), _ranges(case["expect_b"])), case
        elif kind == "conflict":
            want = [(s["start"], s["end"], f) for s, f in reversed(case["expect_spans"])]
            assert ans == (want, case["expect_common"]), case
        else:
            assert ans == case["expected"], case


def _hist_of(name):
    o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
    ent, po, par = o.export("entries"), o.export("parent_offsets"), o.export("parents")
    return [{"span": [int(s), int(e)], "parents": [int(p) for p in par[po[k]:po[k + 1]]]}
            for k, (s, e) in enumerate(ent)], len(o)


@pytest.mark.parametrize("name", G.DT_FILES)
def test_random_queries_vs_oracle(name):
    hist, n = _hist_of(name)
    og = OracleGraph(hist)
    rng = random.Random(1234)
    queries = []
    for _ in range(300):
        a = sorted(rng.sample(range(n), rng.choice([1, 1, 2])))
        b = sorted(rng.sample(range(n), rng.choice([1, 1, 2])))
        queries.append(("diff", 0, a, b))
        queries.append(("conflict", 0, a, b))
        queries.append(("contains", 0, a, rng.randrange(-1, n)))
    got = dt_amd.graph_queries([hist], queries, span_cap=4096)
    checked = 0
    for (kind, _g, a, b), ans in zip(queries, got):
        # no capacity limit: a queue that outgrows LDS is answered again from HBM scratch
        assert not (isinstance(ans, tuple) and ans and ans[0] == "error"), (kind, a, b, ans)
        if kind == "diff":
            oa, ob = og.diff(a, b)
            assert ans == (list(reversed(oa)), list(reversed(ob))), (a, b)
        elif kind == "conflict":
            assert ans == og.find_conflicting(a, b), (a, b)
        else:
            assert ans == og.contains(a, b), (a, b)
        checked += 1
    assert checked == len(queries)


FANCY = [{"span": [0, 3], "parents": []}, {"span": [3, 6], "parents": []},
         {"span": [6, 9], "parents": [1, 4]}, {"span": [9, 11], "parents": [2, 8]}]
# dominator_smoke_test (tools.rs:1030-1051)
DOMINATOR_KATS = [([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10], [5, 10]), ([10], [10]), ([5, 6], [5, 6]), ([5, 9], [5, 9]),
                  ([4, 9], [9]), ([1, 2], [2]), ([0, 2], [2]), ([0, 10], [10]), ([], []), ([2], [2]),
                  ([1, 4], [1, 4]), ([9, 10], [10]), ([2, 8, 9], [9]), ([2, 7, 9], [9]), ([6, 7], [7]), ([0], [0])]


def test_dominator_kats_one_batch():
    """find_dominators_2 on the device for every split of every dominator_smoke_test input into
    two dominator sets, both orders (check_dominators, tools.rs:993-1028)."""
    og = OracleGraph(FANCY)
    queries, want = [], []
    for inp, exp in DOMINATOR_KATS:
        for k in range(len(inp) + 1):
            a, b = og.dominators(inp[:k]), og.dominators(inp[k:])
            queries += [("dominators", 0, a, b), ("dominators", 0, b, a)]
            want += [exp, exp]
    assert dt_amd.graph_queries([FANCY], queries) == want


@pytest.mark.parametrize("name", G.DT_FILES)
def test_random_dominators_vs_oracle_and_host(name):
    """Device find_dominators_2 of random dominator-set pairs over the benchmark graphs against
    the oracle's definition (no member in another's history) and the host engine's."""
    hist, n = _hist_of(name)
    og = OracleGraph(hist)
    o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
    rng = random.Random(77)
    queries = []
    for _ in range(400):
        a = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2, 3]))))
        b = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2, 3]))))
        queries.append(("dominators", 0, a, b))
    got = dt_amd.graph_queries([hist], queries)
    for (_k, _g, a, b), ans in zip(queries, got):
        want = og.dominators(a, b)
        assert ans == want, (a, b)
        assert o.dominators(a, b) == want, (a, b)


def test_level_synchronous_diff_fixtures():
    """Graph::diff by level-synchronous propagation (dt_level.hip) on every diff.json fixture."""
    graphs, queries, cases = [], [], []
    for case in G.cg_fixture("diff"):
        graphs.append(case["hist"])
        queries.append(("diff_level", len(graphs) - 1, case["a"], case["b"]))
        cases.append(case)
    for case, ans in zip(cases, dt_amd.graph_queries(graphs, queries)):
        assert ans == (_ranges(case["expect_a"]), _ranges(case["expect_b"])), case


@pytest.mark.parametrize("name", G.DT_FILES)
def test_level_synchronous_diff_vs_heap_walk_and_oracle(name):
    """The level sweep and the heap walk give the same span lists on random version pairs of the
    benchmark graphs (one batch holding both kinds), and both equal the oracle's diff."""
    hist, n = _hist_of(name)
    og = OracleGraph(hist)
    rng = random.Random(4321)
    pairs = []
    for _ in range(150):
        a = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2]))))
        b = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2]))))
        pairs.append((a, b))
    queries = [("diff_level", 0, a, b) for a, b in pairs] + [("diff", 0, a, b) for a, b in pairs]
    got = dt_amd.graph_queries([hist], queries, span_cap=4096)
    lev, heap = got[:len(pairs)], got[len(pairs):]
    for (a, b), x, y in zip(pairs, lev, heap):
        oa, ob = og.diff(a, b)
        assert x == (list(reversed(oa)), list(reversed(ob))), (a, b)
        if not (isinstance(y, tuple) and y and y[0] == "error"):
            assert x == y, (a, b)


def test_level_synchronous_conflict_fixtures():
    """Graph::find_conflicting by level-synchronous marks + the bucketed sweep (dt_level.hip) on
    every conflicting.json fixture (tools.rs:779-901 semantics)."""
    graphs, queries, cases = [], [], []
    for case in G.cg_fixture("conflicting"):
        graphs.append(case["hist"])
        queries.append(("conflict_level", len(graphs) - 1, case["a"], case["b"]))
        cases.append(case)
    for case, ans in zip(cases, dt_amd.graph_queries(graphs, queries)):
        want = [(s["start"], s["end"], f) for s, f in reversed(case["expect_spans"])]
        assert ans == (want, case["expect_common"]), case


@pytest.mark.parametrize("name", G.DT_FILES)
def test_level_conflict_random_vs_oracle_and_heap_walk(name):
    hist, n = _hist_of(name)
    og = OracleGraph(hist)
    rng = random.Random(4321)
    pairs = []
    for _ in range(300):
        a = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2, 3]))))
        b = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2, 3]))))
        pairs.append((a, b))
    queries = [("conflict_level", 0, a, b) for a, b in pairs] + [("conflict", 0, a, b) for a, b in pairs]
    got = dt_amd.graph_queries([hist], queries, span_cap=8192)
    lvl, heap = got[:len(pairs)], got[len(pairs):]
    for (a, b), x, y in zip(pairs, lvl, heap):
        assert x == og.find_conflicting(a, b), (a, b)
        assert x == y, (a, b)   # the heap walk has no queue limit either


def _wide_history(n_entries, seed):
    """Two agents taking turns, each entry a 2-LV run whose parents are the dominators of the
    agent's own last LV and a random recent LV of the other's (oracle Graph::find_dominators)."""
    rng = random.Random(seed)
    og = OracleGraph()
    hist, last = [], [None, None]
    for i in range(n_entries):
        who = i % 2
        cand = [x for x in (last[who],) if x is not None]
        if last[1 - who] is not None and rng.random() < 0.7:
            cand.append(max(0, last[1 - who] - 2 * rng.randrange(3)))
        parents = og.dominators(sorted(set(cand))) if cand else []
        og.push(parents, 2 * i, 2 * i + 2)
        hist.append({"span": [2 * i, 2 * i + 2], "parents": parents})
        last[who] = 2 * i + 1
    return hist, og


def test_level_kernels_past_the_old_lds_cap():
    """12,000 entries (the round-2 level kernels held per-entry state in LDS, capped at 8,192):
    level-synchronous diff and conflict spans against the oracle."""
    hist, og = _wide_history(12000, 7)
    n = 24000
    rng = random.Random(9)
    pairs = []
    for _ in range(40):
        a = og.dominators(sorted(rng.sample(range(n), rng.choice([1, 2]))))
        b = og.dominators(sorted(rng.sample(range(n // 2), rng.choice([1, 2]))))
        pairs.append((a, b))
    queries = [("diff_level", 0, a, b) for a, b in pairs] + [("conflict_level", 0, a, b) for a, b in pairs]
    got = dt_amd.graph_queries([hist], queries, span_cap=32768)
    for (a, b), d, c in zip(pairs, got[:len(pairs)], got[len(pairs):]):
        oa, ob = og.diff(a, b)
        assert d == (list(reversed(oa)), list(reversed(ob))), (a, b)
        assert c == og.find_conflicting(a, b), (a, b)


def _fan_history(width, depth, seed):
    """`width` concurrent branches from ROOT (3-LV entries, `depth` deep), then one entry merging
    every branch tip (`width` parents), then a few more concurrent branches off the merge: wide
    frontiers, a wide merge point and a queue far past the LDS heaps' 256 keys / 64 time points."""
    rng = random.Random(seed)
    og = OracleGraph()
    hist, tips, lv = [], [], 0
    for w in range(width):
        prev = []
        for d in range(depth):
            og.push(prev, lv, lv + 3)
            hist.append({"span": [lv, lv + 3], "parents": prev})
            prev = [lv + 2]
            lv += 3
        tips.append(prev[0])
    og.push(sorted(tips), lv, lv + 2)
    hist.append({"span": [lv, lv + 2], "parents": sorted(tips)})
    merge = lv + 1
    lv += 2
    tails = []
    for w in range(width // 2):
        p = [merge] if w % 2 == 0 else [rng.choice(tips)]
        og.push(p, lv, lv + 2)
        hist.append({"span": [lv, lv + 2], "parents": p})
        tails.append(lv + 1)
        lv += 2
    return hist, og, tips, tails, lv


@pytest.mark.parametrize("width", [24, 80])
def test_wide_frontiers_and_merges_vs_oracle(width):
    """Frontiers of 20-80 versions, a merge of `width` parents and queues past the LDS heaps: every
    heap-walk and level-synchronous query against the oracle, none reporting capacity."""
    hist, og, tips, tails, n = _fan_history(width, 4, width)
    rng = random.Random(7)
    queries = []
    for _ in range(30):
        a = og.dominators(sorted(rng.sample(tips, rng.randint(1, min(len(tips), 40)))))   # concurrent: wide
        b = og.dominators(sorted(rng.sample(tips + tails, rng.randint(1, min(len(tips), 40)))))
        for kind in ("diff", "conflict", "dominators", "diff_level", "conflict_level"):
            queries.append((kind, 0, a, b))
        queries.append(("contains", 0, a, rng.randrange(-1, n)))
    got = dt_amd.graph_queries([hist], queries, span_cap=16384)
    assert any(len(q[2]) > 16 for q in queries)
    for (kind, _g, a, b), ans in zip(queries, got):
        assert not (isinstance(ans, tuple) and ans and ans[0] == "error"), (kind, len(a), ans)
        if kind in ("diff", "diff_level"):
            oa, ob = og.diff(a, b)
            assert ans == (list(reversed(oa)), list(reversed(ob))), (kind, a, b)
        elif kind in ("conflict", "conflict_level"):
            assert ans == og.find_conflicting(a, b), (kind, a, b)
        elif kind == "dominators":
            assert ans == og.dominators(sorted(set(a) | set(b))), (a, b)
        else:
            assert ans == og.contains(a, b), (a, b)
