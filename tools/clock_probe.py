"""In-kernel clock and document timeline of the replay (lib_clock variant build: every document
stamps s_memtime / s_memrealtime at its start and end into its result's debug words).
  DTGPU_LIB_DIR=lib_clock python tools/clock_probe.py friendsforever 10000"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import dt_amd
    import golden_data as G
    name, n = sys.argv[1], int(sys.argv[2])
    b = dt_amd.Batch(docs=[G.dt_bytes(name)] * n, staging="device")
    b.run(); b.sync()
    for _ in range(3):
        ms = b.run_timed()
    st = [b.doc_stats(i) for i in range(n)]
    while True:   # the segment documents after them
        try:
            st.append(b.doc_stats(len(st)))
        except Exception:
            break
    n = len(st)
    mt = np.array([s["cyc_ins"] for s in st], dtype=np.float64)
    rt = np.array([s["cyc_del"] for s in st], dtype=np.float64)
    t0 = np.array([s["cyc_tog"] for s in st], dtype=np.int64)
    t1 = np.array([s["cyc_mat"] for s in st], dtype=np.int64)
    base = t0.min()
    start_ms, end_ms = (t0 - base) / 1e5, (t1 - base) / 1e5
    ghz = mt / rt / 10.0
    print(f"{name} x{n}: pass {ms:.2f} ms; clock median {np.median(ghz):.3f} GHz (p10 {np.percentile(ghz, 10):.3f}, "
          f"p90 {np.percentile(ghz, 90):.3f}); doc duration ms median {np.median(rt) / 1e5:.2f} "
          f"min {rt.min() / 1e5:.2f} max {rt.max() / 1e5:.2f}; replay span {end_ms.max():.2f} ms")
    order = np.argsort(start_ms)
    for q in (0, 0.25, 0.5, 0.75, 0.8, 0.85, 0.9, 0.95, 1.0):
        k = order[min(n - 1, int(q * (n - 1)))]
        print(f"  doc started at quantile {q:.2f}: start {start_ms[k]:.2f} ms, end {end_ms[k]:.2f} ms, "
              f"duration {(end_ms[k] - start_ms[k]):.2f} ms")
    hist = np.histogram(start_ms, bins=20)
    print("  start-time histogram:", list(hist[0]), "edges ms", [round(x, 1) for x in hist[1][::4]])




def by_unit(name="friendsforever", n=10000):
    """Durations of the documents that started at once, grouped by XCD / SE / CU / SIMD."""
    import numpy as np
    import dt_amd
    import golden_data as G
    b = dt_amd.Batch(docs=[G.dt_bytes(name)] * n, staging="device")
    b.run(); b.sync()
    b.run_timed()
    st = [b.doc_stats(i) for i in range(n)]
    while True:   # the segment documents after them
        try:
            st.append(b.doc_stats(len(st)))
        except Exception:
            break
    n = len(st)
    rt = np.array([s["cyc_del"] for s in st], dtype=np.float64) / 1e5
    t0 = np.array([s["cyc_tog"] for s in st], dtype=np.int64)
    hw = np.array([s["cyc_yjs"] for s in st], dtype=np.int64)
    xcc = np.array([s["cyc_split"] for s in st], dtype=np.int64) & 7
    first = (t0 - t0.min()) < 100   # started within 1 us of the first
    simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
    for label, key in (("xcc", xcc), ("se", se), ("simd", simd)):
        vals = {int(k): (round(float(np.median(rt[first & (key == k)])), 2), int((first & (key == k)).sum()))
                for k in np.unique(key[first])}
        print(f"  first batch by {label}: median ms (docs) {vals}")
    cid = xcc * 128 + se * 16 + cu
    per = {int(k): float(np.median(rt[first & (cid == k)])) for k in np.unique(cid[first])}
    v = np.array(list(per.values()))
    print(f"  per-CU median duration: min {v.min():.2f} p25 {np.percentile(v, 25):.2f} median {np.median(v):.2f} "
          f"p75 {np.percentile(v, 75):.2f} max {v.max():.2f} over {len(v)} CUs")
    later = ~first
    cnt = {int(k): int((later & (cid == k)).sum()) for k in np.unique(cid)}
    c = np.array(list(cnt.values()))
    print(f"  later documents per CU: max {c.max()} mean {c.mean():.1f} CUs with any {int((c > 0).sum())}")
    wave_pos = hw & 15
    print(f"  first batch by wave slot: {dict((int(k), round(float(np.median(rt[first & (wave_pos == k)])), 2)) for k in np.unique(wave_pos[first]))}")


if __name__ == "__main__":
    if sys.argv[1] == "--units":
        by_unit(sys.argv[2], int(sys.argv[3]))
    else:
        main()
