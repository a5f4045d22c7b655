"""Single-document `.dt` decode time of each configs[4] trace (the 3 .dt files and the 5 JSON
traces written as .dt), to find which one bounds a mixed batch's decode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402

docs = [(n, G.dt_bytes(n)) for n in G.DT_FILES]
docs += [(n, dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode()) for n in G.JSON_TRACES]
for name, data in docs:
    one = dt_amd.DecodeBatch([data])
    one.run()
    ms = min(one.run() for _ in range(3))
    o = dt_amd.ListOpLog.load_from(data)
    print(f"{name}: {len(data)} B, {len(o)} LVs, {len(o.export('ops'))} op runs, decode {ms:.2f} ms; "
          f"phases {one.profile(0)}", flush=True)

# device encoder, one document alone per trace (ENCODE_FULL; bytes checked against the host)
if os.environ.get("DMIXED_ENCODE"):
    for name, data in docs:
        b = dt_amd.Batch(docs=[data], staging="device")
        ms = min(b.encode() for _ in range(3))
        ok = b.encoded(0) == dt_amd.ListOpLog.load_from(data).encode()
        print(f"{name}: encode {ms:.2f} ms, bytes equal host: {ok}", flush=True)
