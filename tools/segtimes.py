"""Per-segment replay times of one cut document (lib_clock build: each document stamps its
start / end and command count into its debug words).  DTGPU_LIB_DIR=lib_clock python tools/segtimes.py NAME"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    name = sys.argv[1]
    data = G.dt_bytes(name) if name in G.DT_FILES else dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
    b = dt_amd.Batch(docs=[data], staging="device")
    b.run(); b.sync()
    ms = min(b.run_timed() for _ in range(3))
    segs = [(g["lo"], g["hi"], g["placeholders"]) for g in b.segments(0)]
    st = []
    while True:
        try:
            st.append(b.doc_stats(len(st)))
        except Exception:
            break
    t0 = min(s["cyc_tog"] for s in st)
    print(f"{name}: pass {ms:.2f} ms, {len(st)} segment documents")
    if os.environ.get("DTGPU_DEBUG") == "2":   # cycle profile (main build): phases in M cycles
        for i, s in enumerate(st):
            print(f"  seg doc {i}: " + " ".join(f"{k[4:]} {s[k] * 16 / 1e6:.2f}" for k in
                  ("cyc_ins", "cyc_del", "cyc_tog", "cyc_mat", "cyc_split", "cyc_find", "cyc_bload", "cyc_total"))
                  + f" splits {s['n_split']} blocks {s['n_blocks']} items {s['n_items']} cmds {s['n_cmds']}")
        return
    for i, s in enumerate(st):
        print(f"  seg doc {i}: start {(s['cyc_tog'] - t0) / 1e5:6.2f} ms  dur {s['cyc_del'] / 1e5:6.2f} ms  "
              f"cmds {s['cyc_yjs']}  lvs {s['cyc_split']}")
    print("  ranges:", segs)


if __name__ == "__main__":
    main()
