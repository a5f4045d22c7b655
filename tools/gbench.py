"""Batched causal-graph query throughput (dt_graph.hip): random diff / find_conflicting /
version_contains queries over a benchmark file's graph.  Usage: python tools/gbench.py [name] [n]"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "node_nodecc"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
ent, po, par = o.export("entries"), o.export("parent_offsets"), o.export("parents")
hist = [{"span": [int(s), int(e)], "parents": [int(p) for p in par[po[k]:po[k + 1]]]} for k, (s, e) in enumerate(ent)]
rng = random.Random(5)
nl = len(o)
for kind in ("diff", "conflict", "contains"):
    qs = []
    for _ in range(n):
        a = sorted(rng.sample(range(nl), 1 + (rng.random() < 0.3)))
        b = sorted(rng.sample(range(nl), 1 + (rng.random() < 0.3))) if kind != "contains" else rng.randrange(nl)
        qs.append((kind, 0, a, b))
    dt_amd.graph_queries([hist], qs[:64], span_cap=4096)
    out, ms = dt_amd.graph_queries([hist], qs, span_cap=4096, timing=True)
    errs = sum(1 for x in out if isinstance(x, tuple) and x and x[0] == "error")
    print(f"{name} {kind}: {n} queries in {ms:.2f} ms = {n / ms * 1e3 / 1e6:.2f} M queries/s (capacity stops {errs})",
          flush=True)
