"""Step-by-step GPU probe with flushed progress lines (debug aid for gpurun sessions)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    import dt_amd
    import golden_data as G
    from oracle.oracle import OpLog as OO
    log("devices", dt_amd.device_count())
    which = sys.argv[1:] or ["compat", "friendsforever"]
    for w in which:
        if w == "compat":
            data = G.COMPAT_SIMPLE_LZ4
        else:
            data = G.dt_bytes(w)
        t = time.time()
        o = dt_amd.ListOpLog.load_from(data)
        log(w, "loaded", len(o), o.plan_stats())
        got = o.checkout_tip_bytes()
        log(w, "gpu checkout", len(got), f"{time.time() - t:.3f}s")
        want = OO.load_from(data).checkout_tip_bytes()
        log(w, "match" if got == want else f"MISMATCH want {len(want)}")
        if got != want:
            n = min(len(got), len(want))
            i = next((k for k in range(n) if got[k] != want[k]), n)
            log("first diff at", i, got[max(0, i - 40):i + 40], want[max(0, i - 40):i + 40])


if __name__ == "__main__":
    main()
