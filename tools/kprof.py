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
        if name.startswith("synth"):   # synth[:distinct]x<copies>: pairwise-merge synthetic docs
            distinct = int(name.split(":")[1]) if ":" in name else 64
            pool = [dt_amd.synth_merge_oplog(i, 5000).encode() for i in range(distinct)]
            b = dt_amd.Batch(docs=[pool[i % distinct] for i in range(copies)], staging="device")
        else:
            b = dt_amd.Batch(docs=[G.dt_bytes(name)] * copies, staging="device")
        ms = b.run_timed()
        idx = range(0, copies, max(1, copies // 16))
        sts = [b.doc_stats(i) for i in idx]
        st = {k: sum(x[k] for x in sts) // len(sts) for k in sts[0]}
        res = b.results()[0]
        cyc = {k: v * 16 for k, v in st.items() if k.startswith("cyc_")}
        tot = max(1, cyc["cyc_total"])
        parts = " ".join(f"{k[4:]}={v / 1e6:.2f}M({100 * v / tot:.0f}%)" for k, v in cyc.items())
        print(f"{name}x{copies}: status={res['status']} ms={ms:.2f} cmds={st['n_cmds']} items={st['n_items']} "
              f"blocks={st['n_blocks']}/{st['max_blocks']} sb={st['n_sb']} lds={st['lds_index']} yjs={st['n_yjs']} splits={st['n_split']} "
              f"loads={st['n_load']} dirty={st['n_dirty']} {parts}",
              flush=True)
        for k, s in enumerate(b.segments(0)):   # cut replay: one wave per segment
            print(f"  segment {k}: lv [{s['lo']}, {s['hi'] if s['hi'] != 0xFFFFFFFF else 'end'}) "
                  f"placeholders={s['placeholders']} visible={s['items_visible']} "
                  f"cycles={s['cyc_total'] * 16 / 1e6:.2f}M lds={s['lds_index']} blocks={s['n_blocks']}", flush=True)




def plan_profile(names):
    """Planner cycle profile (DTGPU_PLAN_PROF): python tools/kprof.py --plan friendsforever ..."""
    os.environ["DTGPU_PLAN_PROF"] = "1"
    import dt_amd
    import golden_data as G
    for a in names:
        name, _, copies = a.partition("x")
        copies = int(copies or 1)
        b = dt_amd.Batch(docs=[G.dt_bytes(name)] * copies, staging="device")
        b.run_timed()
        ms = b.last_times()
        pr = [b.plan_profile(i) for i in range(0, copies, max(1, copies // 16))]
        avg = {k: sum(x[k] for x in pr) / len(pr) for k in pr[0]}
        tot = sum(avg[k] for k in ("rec", "parents", "children", "emit", "ops", "init"))
        print(f"{a}: plan_ms={ms[0]:.2f} " + " ".join(f"{k}={avg[k] / 1e6:.2f}M({100 * avg[k] / max(tot, 1):.0f}%)"
                                                     for k in ("rec", "parents", "children", "emit", "ops", "init"))
              + f" cmds={avg['n_cmds']:.0f} tlist={avg['n_tlist']:.0f}", flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--plan"]:
        plan_profile(sys.argv[2:])
    else:
        main()
