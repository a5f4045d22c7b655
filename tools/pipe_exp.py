"""Pass time of 10,000 friendsforever documents split into k device-staged batches launched on
their own streams back to back (prep -> plan -> replay per batch): do the batches' kernels fill
each other's tails?  usage: python tools/pipe_exp.py [name] [docs] [k,k,...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "friendsforever"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    ks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,3,4").split(",")]
    data = G.dt_bytes(name)
    for k in ks:
        sizes = [n // k + (1 if i < n % k else 0) for i in range(k)]
        bs = [dt_amd.Batch(docs=[data] * s, staging="device") for s in sizes]
        for _ in range(2):
            for b in bs:
                b.run()
            for b in bs:
                b.sync()
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            for b in bs:
                b.run()
            for b in bs:
                b.sync()
            best = min(best, (time.perf_counter() - t0) * 1e3)
        ok = all(b.results()[0]["status"] == 0 and b.results()[-1]["text_hash"] == bs[0].results()[0]["text_hash"]
                 for b in bs)
        print(f"{name} x{n} in {k} batches {sizes}: {best:.2f} ms per pass (wall, launch + sync) ok={ok}", flush=True)
        del bs


if __name__ == "__main__":
    main()
