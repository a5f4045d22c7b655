"""Instruction mix per command type of the replay: synthetic single-agent documents (typing runs
only; typing runs + backspace / forward delete runs) beside friendsforever, each replayed as a
10,000-copy batch with cut replay off, so that PMC instruction counts (SQ_INSTS_*) divided by the
commands give each command type's cost.  Run under rocprofv3 --pmc (tools/r5h.sh).
  DTGPU_SEG=0 python tools/salu_probe.py ins|insdel|friendsforever [copies]"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def typing_doc(n_runs, with_deletes, seed=7):
    """One agent typing: runs of ~7 chars, each one char before the previous run's end (so runs stay
    separate commands, as two interleaved authors' are), the cursor sometimes jumping;
    with_deletes: every 6th run is a delete run (backspace or forward) near the cursor."""
    import dt_amd
    rnd = random.Random(seed)
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("typist")
    length, cur = 0, 0
    for k in range(n_runs):
        if rnd.random() < 0.1:
            cur = rnd.randint(0, length)
        if with_deletes and k % 6 == 5 and length > 8:
            n = rnd.randint(1, 4)
            if rnd.random() < 0.5 and cur >= n:   # backspace
                o.add_delete_without_content(a, cur - n, cur)
                cur -= n
            else:
                s = min(cur, length - n)
                o.add_delete_without_content(a, s, s + n)
                cur = s
            length -= n
            continue
        n = rnd.randint(3, 11)
        o.add_insert(a, cur, "".join(rnd.choice("abcdefghij ") for _ in range(n)))
        cur += n - 1   # the next run starts one char back: a separate op run (as interleaved typing)
        length += n
    return o.encode()


def main():
    import dt_amd
    import golden_data as G
    kind = sys.argv[1]
    copies = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    if kind == "friendsforever":
        data = G.dt_bytes("friendsforever")
    else:
        data = typing_doc(3900 if kind == "insdel" else 3342, kind == "insdel")
    o = dt_amd.ListOpLog.load_from(data)
    st = o.plan_stats()
    b = dt_amd.Batch(docs=[data] * copies, staging="device")
    b.run(); b.sync()
    ms = b.run_timed()
    res = b.results()
    assert all(r["status"] == 0 for r in res)
    assert all(b.segments(i) == [] for i in range(0, copies, 1000))
    pl = o.plan_commands()
    kinds = {"ins": 0, "del": 0, "tog": 0}
    for c in pl:
        kinds[("ins", "del", "tog")[int(c[0]) & 15]] += 1
    print(f"{kind} x{copies}: kernel {ms:.2f} ms replay {b.last_times()[1]:.2f} ms; LVs {len(o)}; plan {st}; commands {kinds}",
          flush=True)


if __name__ == "__main__":
    main()
