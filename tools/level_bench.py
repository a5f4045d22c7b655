"""Heap-walk diff / find_conflicting (dt_graph.hip, one wavefront per query) vs the
level-synchronous forms (dt_level.hip: levelling + one workgroup per query) on the same random version pairs of the
configs[2] graphs (node_nodecc, git-makefile) and friendsforever.  Device time of one batch,
levelling included in the level-synchronous figure; a one-query batch gives the levelling cost."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for name in ("node_nodecc", "git-makefile", "friendsforever"):
        o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
        ent, po, par = o.export("entries"), o.export("parent_offsets"), o.export("parents")
        hist = [{"span": [int(s), int(e)], "parents": [int(p) for p in par[po[k]:po[k + 1]]]}
                for k, (s, e) in enumerate(ent)]
        n = len(o)
        rng = random.Random(9)
        pairs = [(o.dominators(sorted(rng.sample(range(n), rng.choice([1, 2])))),
                  o.dominators(sorted(rng.sample(range(n), rng.choice([1, 2]))))) for _ in range(nq)]
        res = {}
        for kind in ("diff", "diff_level", "conflict", "conflict_level"):
            best = None
            for _ in range(3):
                out, ms = dt_amd.graph_queries([hist], [(kind, 0, a, b) for a, b in pairs], span_cap=4096, timing=True)
                best = ms if best is None else min(best, ms)
            res[kind] = (best, out)
        one = min(dt_amd.graph_queries([hist], [("diff_level", 0, *pairs[0])], timing=True)[1] for _ in range(3))
        same = sum(1 for x, y in zip(res["diff"][1], res["diff_level"][1]) if x == y)
        csame = sum(1 for x, y in zip(res["conflict"][1], res["conflict_level"][1]) if x == y)
        print(f"{name}: entries={len(hist)} queries={nq} diff: heap_walk_ms={res['diff'][0]:.3f} "
              f"level_sync_ms={res['diff_level'][0]:.3f} (levelling+1 query {one:.3f} ms) agree={same}/{nq}; "
              f"conflict: heap_walk_ms={res['conflict'][0]:.3f} level_sync_ms={res['conflict_level'][0]:.3f} "
              f"agree={csame}/{nq}", flush=True)


if __name__ == "__main__":
    main()
