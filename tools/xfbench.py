"""Transformed-ops (iter_xf_operations, src/list/merge.rs:40-48) batch benchmark: N copies of a
`.dt` document staged as one xf batch (dtgpu_batch_create_xf), device passes timed with HIP
events, every document's per-LV BaseMoved positions checked against the C oracle's (which the
tests pin to the reference's own export of friendsforever).  Prints one JSON line.

usage: python tools/xfbench.py [name] [docs] [reps]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    from oracle.oracle import OpLog as OracleOpLog
    name = sys.argv[1] if len(sys.argv) > 1 else "friendsforever"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    data = G.dt_bytes(name)
    ora = OracleOpLog.load_from(data)
    want = {lv: (None if x < 0 else x) for lv, x in ora.xf_operations()}
    one = dt_amd.ListOpLog.load_from(data)
    t0 = time.time()
    b = dt_amd.Batch(oplogs=[one] * n, xf=True)
    stage = time.time() - t0
    b.run()
    b.sync()
    ms = [b.run_timed() for _ in range(reps)]
    res = b.results()
    assert all(r["status"] == 0 for r in res)
    check = sorted({0, n // 2, n - 1})
    for i in check:
        got = b.xf_positions(i)
        assert all(got[lv] == x for lv, x in want.items()), f"doc {i} differs from the oracle"
    lv = sum(r["n_lv"] for r in res)
    mean = statistics.mean(ms)
    print(json.dumps({"workload": f"{name} x {n} docs (iter_xf_operations, transformed-ops replay)",
                      "kernel_ms": mean, "all_ms": ms, "xf_ops_per_s": lv / (mean / 1000.0),
                      "docs_per_s": n / (mean / 1000.0), "stage_s": stage,
                      "checked_docs": check, "parity": "per-LV BaseMoved positions == C oracle"}), flush=True)


if __name__ == "__main__":
    main()
