"""Replay one document (optionally with DTGPU_DEBUG=1 invariant checks) and print the failing
command and code site.  python tools/span_debug.py git-makefile [debug]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
if len(sys.argv) > 2:
    os.environ["DTGPU_DEBUG"] = sys.argv[2]


def main():
    import dt_amd
    import golden_data as G
    data = G.dt_bytes(sys.argv[1])
    for staging in ("host", "device"):
        b = dt_amd.Batch(docs=[data], staging=staging)
        b.run()
        b.sync()
        r = b.results()[0]
        st = b.doc_stats(0)
        print(staging, r, {k: st[k] for k in ("n_items", "n_blocks", "fail_cmd", "fail_site", "n_cmds", "max_blocks", "n_sb", "lds_index")}, flush=True)
        if r["status"] != 0:
            op = dt_amd.ListOpLog.load_from(data)
            cmds = op.plan_commands()
            fc = st["fail_cmd"]
            print("commands around the failure:", cmds[max(0, fc - 3):fc + 2])


if __name__ == "__main__":
    main()
