"""Kernel-time micro-benchmark: stage N copies of a document and time device passes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    name = sys.argv[1]
    counts = [int(x) for x in sys.argv[2].split(",")]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    distinct = None
    if name.startswith("synth"):   # synth[:distinct] -- synthetic concurrent docs (dt_synth.cpp)
        distinct = int(name.split(":")[1]) if ":" in name else 256
        pool = [dt_amd.synth_merge_oplog(i, 5000) for i in range(distinct)]
    elif name in G.JSON_TRACES:   # a linear trace, built as crates/bench builds it, written as .dt
        data = dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
    else:
        data = G.dt_bytes(name)
    for n in counts:
        t = time.time()
        if distinct:
            b = dt_amd.Batch(oplogs=[pool[i % distinct] for i in range(n)])
        else:
            b = dt_amd.Batch(docs=[data] * n, staging="device")
        stage = time.time() - t
        b.run(); b.sync()
        ms, split = [], []
        for _ in range(reps):
            ms.append(b.run_timed())
            split.append(b.last_times())
        res = b.results()
        ok = all(r["status"] == 0 for r in res)
        lv = sum(r["n_lv"] for r in res)
        best = min(ms)
        print(f"{name} docs={n} stage={stage:.2f}s kernel_ms={best:.2f} (all {['%.2f' % m for m in ms]}) "
              f"ok={ok} Mops/s={lv / best / 1e3:.1f} alg_GB/s={b.algorithmic_bytes / best / 1e6:.1f} "
              f"plan/replay_ms={split[ms.index(best)][0]:.2f}/{split[ms.index(best)][1]:.2f} host_planned={sum(b.host_planned())} "
              f"ff={sum(b.fast_forwarded())}",
              flush=True)


if __name__ == "__main__":
    main()
