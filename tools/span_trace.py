"""DTGPU_DEBUG=8: the replay writes the visible total after every command instead of the text;
dump them (one per line) for comparison with a model.  python tools/span_trace.py git-makefile out.txt"""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["DTGPU_DEBUG"] = "8"

import dt_amd
import golden_data as G

b = dt_amd.Batch(docs=[G.dt_bytes(sys.argv[1])], staging="host")
b.run()
b.sync()
raw = b.text(0)
vals = struct.unpack("<%dI" % (len(raw) // 4), raw[:len(raw) // 4 * 4])
open(sys.argv[2], "w").write("\n".join(map(str, vals)) + "\n")
print("status", b.results()[0]["status"], "fail_cmd", b.doc_stats(0)["fail_cmd"], "n", len(vals))
