"""Replay timeline of the mixed workload by trace (lib_clock variant build: every document stamps
its start / end into its debug words).  DTGPU_LIB_DIR=lib_clock python tools/mixed_probe.py"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(n_docs=400):
    import numpy as np
    import dt_amd
    import golden_data as G
    names = list(G.DT_FILES) + list(G.JSON_TRACES)
    datas = [G.dt_bytes(n) if n in G.DT_FILES else dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode()
             for n in names]
    b = dt_amd.Batch(docs=[datas[i % 8] for i in range(n_docs)], staging="device")
    b.run(); b.sync()
    print("pass ms", min(b.run_timed() for _ in range(3)))
    st = []
    while True:
        try:
            st.append(b.doc_stats(len(st)))
        except Exception:
            break
    t0 = min(s["cyc_tog"] for s in st)
    by = collections.defaultdict(list)
    for i, s in enumerate(st):
        by[names[i % 8] if i < n_docs else "segments"].append(((s["cyc_tog"] - t0) / 1e5, s["cyc_del"] / 1e5,
                                                               s["cyc_ins"] / max(s["cyc_del"], 1) / 10.0))
    for k, v in by.items():
        a = np.array(v)
        end = a[:, 0] + a[:, 1]
        print(f"{k:20s} n {len(v):4d} start min/med/max {a[:, 0].min():6.2f} {np.median(a[:, 0]):6.2f} "
              f"{a[:, 0].max():6.2f}  dur med/max {np.median(a[:, 1]):6.2f} {a[:, 1].max():6.2f}  end max {end.max():6.2f}"
              f"  clock {np.median(a[:, 2]):.2f} GHz")


if __name__ == "__main__":
    main()
