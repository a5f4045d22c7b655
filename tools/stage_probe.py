"""Cold-path staging probe: wall time of Batch(docs=..., staging="device") for N copies of a
document, with the library's per-phase clock (DTGPU_STAGE_PROF=1), then one pass.
Usage: DTGPU_STAGE_PROF=1 python tools/stage_probe.py friendsforever 10000"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    name, n = sys.argv[1], int(sys.argv[2])
    data = G.dt_bytes(name) if name in G.DT_FILES else dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
    docs = [bytes(data) for _ in range(n)]
    dt_amd.device_count()
    warm = dt_amd.Batch(docs=docs[:2], staging="device")   # the HIP runtime and code objects, loaded once
    del warm
    for rep in range(2):
        t0 = time.perf_counter()
        b = dt_amd.Batch(docs=docs, staging="device")
        t1 = time.perf_counter()
        ms = b.run_timed()
        b.sync()
        t2 = time.perf_counter()
        ok = all(r["status"] == 0 for r in b.results())
        print(f"{name} x {n}: staging {1e3 * (t1 - t0):.1f} ms, first pass {ms:.2f} ms (wall {1e3 * (t2 - t1):.1f} ms), "
              f"cold total {1e3 * (t2 - t0):.1f} ms, ok={ok}", flush=True)
        del b


if __name__ == "__main__":
    main()
