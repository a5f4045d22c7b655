"""GPU `.dt` decode throughput: N copies of a benchmark file, one wavefront per document.
Usage: python tools/dbench.py [name] [docs] [runs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "friendsforever"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 5
data = G.dt_bytes(name)
t0 = time.perf_counter()
dec = dt_amd.DecodeBatch([data] * n)
stage = time.perf_counter() - t0
ms = [dec.run() for _ in range(runs)]
bad = sum(1 for i in range(n) if dec.status(i)["status"] != 0)
best = min(ms)
bi, bo = dec.bytes_in(), dec.bytes_out()
print(f"{name} x{n}: stage {stage:.2f}s decode ms {['%.2f' % m for m in ms]} bad={bad} "
      f"in {bi / best / 1e6:.1f} GB/s in+out {(bi + bo) / best / 1e6:.1f} GB/s "
      f"({bi / n:.0f} B in, {bo / n:.0f} B out per doc)", flush=True)
print("phase cycles doc0 [lz4, chunks, runs, lookup, parents, checks+crc, content+split]:", dec.profile(0))
one = dt_amd.DecodeBatch([data])
one.run()
print(f"single doc: {one.run():.3f} ms; phases {one.profile(0)}", flush=True)
