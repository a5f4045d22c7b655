"""Batched device encoder timing: python tools/encbench.py [doc] [n_docs] [reps]
Prints kernel ms (HIP events), encoded bytes, docs/s, and checks document 0 against the host
encoder."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "diamond-types_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "friendsforever"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
data = G.dt_bytes(name)
docs = [bytes(data) for _ in range(n)]
t0 = time.time()
b = dt_amd.Batch(docs=docs, staging="device")
print(f"staged {n} x {name} in {time.time() - t0:.2f} s", flush=True)
ms = [b.encode() for _ in range(reps)]
host = dt_amd.ListOpLog.load_from(data).encode()
ok = b.encoded(0) == host and b.encoded(n - 1) == host
out_b, in_b = b.encoded_bytes(0), b.encoded_bytes(1)
best = min(ms)
print(f"{name} x {n}: encode kernel ms {['%.2f' % x for x in ms]} best {best:.2f}; out {out_b / 1e6:.1f} MB "
      f"in {in_b / 1e6:.1f} MB; {n / best * 1e3:.0f} docs/s; alg {(out_b + in_b) / best / 1e6:.1f} GB/s; "
      f"bytes equal host: {ok}", flush=True)
if os.environ.get("DTGPU_ENC_PROF"):
    print("profile doc 0:", b.encode_profile(0))
