"""Per-document batch cost of every benchmark trace on the GPU, for the LPT cost model
(dt_amd/shard.py): each trace alone, N device-staged copies, best of 3 passes; prints pass ms / N
with the model's features (LVs, op runs, walk LVs retreated + advanced) as JSON lines.
Usage: python tools/costfit.py [N]"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    for name in list(G.DT_FILES) + list(G.JSON_TRACES):
        if name in G.DT_FILES:
            data = G.dt_bytes(name)
        else:
            data = dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
        o = dt_amd.ListOpLog.load_from(data)
        ps = o.plan_stats()
        runs = len(o.export("ops"))
        b = dt_amd.Batch(docs=[data] * n, staging="device")
        b.run()
        b.sync()
        ms = min(b.run_timed() for _ in range(3))
        ok = all(r["status"] == 0 for r in b.results())
        print(json.dumps({"trace": name, "docs": n, "pass_ms": ms, "ms_per_doc": ms / n, "ok": ok,
                          "lvs": len(o), "runs": runs, "runs_log": runs * math.log2(runs + 1),
                          "walk": ps["retreat"] + ps["advance"]}), flush=True)
        del b


if __name__ == "__main__":
    main()
