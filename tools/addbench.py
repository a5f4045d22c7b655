"""Device decode_and_add throughput (dtgpu_decode_add): N resident copies of a benchmark file's
history at half its length, each merged with (a) the patch after that version (catch-up) and
(b) the whole file (overlap filter).  Prints the merge kernel's ms and documents/s, beside the
host decode_and_add (dt_host.cpp, one thread) on the same pair.

usage: python tools/addbench.py [name] [n_docs]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "diamond-types_amd"))
import golden_data as G  # noqa: E402
import dt_amd  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "friendsforever"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    data = G.dt_bytes(name)
    full = dt_amd.ListOpLog.load_from(data)
    v = full.dominators([len(full) // 2])
    part = full.history(v).encode()
    patch = full.encode_from(v, dt_amd.ENCODE_PATCH)
    d = dt_amd.DecodeBatch([part] * n)
    d.run()
    for label, p in (("catch-up", patch), ("overlap", data)):
        best = None
        for _ in range(3):
            m = d.add([p] * n)
            assert all(m.add_result(i)[0] == 0 for i in (0, n - 1))
            best = m.last_ms if best is None else min(best, m.last_ms)
            del m
        k, host = 20, 0.0
        for _ in range(k):
            h = dt_amd.ListOpLog.load_from(part)
            t0 = time.perf_counter()
            h.decode_and_add(p)
            host += time.perf_counter() - t0
        host_ms = host / k * 1e3
        print(f"{name} {label}: {n} docs, patch {len(p)} B: device merge {best:.2f} ms "
              f"({n / best * 1e3:.0f} docs/s); host decode_and_add {host_ms:.3f} ms/doc "
              f"({1e3 / host_ms:.0f} docs/s, one thread)", flush=True)


if __name__ == "__main__":
    main()
