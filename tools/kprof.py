"""Per-document cycle profile of the replay kernel (DTGPU_DEBUG=2 build path): runs each named
document alone and prints where its wave's time went (s_memtime cycles, /16 on device)."""
import os
import sys

os.environ["DTGPU_DEBUG"] = "2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import dt_amd
    import golden_data as G
    args = sys.argv[1:] or ["friendsforever", "git-makefile", "node_nodecc"]
    for a in args:
        name, _, copies = a.partition("x")
        copies = int(copies or 1)
        b = dt_amd.Batch(docs=[G.dt_bytes(name)] * copies)
        ms = b.run_timed()
        idx = range(0, copies, max(1, copies // 16))
        sts = [b.doc_stats(i) for i in idx]
        st = {k: sum(x[k] for x in sts) // len(sts) for k in sts[0]}
        res = b.results()[0]
        cyc = {k: v * 16 for k, v in st.items() if k.startswith("cyc_")}
        tot = max(1, cyc["cyc_total"])
        parts = " ".join(f"{k[4:]}={v / 1e6:.2f}M({100 * v / tot:.0f}%)" for k, v in cyc.items())
        print(f"{name}x{copies}: status={res['status']} ms={ms:.2f} cmds={st['n_cmds']} items={st['n_items']} "
              f"blocks={st['n_blocks']}/{st['max_blocks']} yjs={st['n_yjs']} splits={st['n_split']} {parts}",
              flush=True)


if __name__ == "__main__":
    main()
