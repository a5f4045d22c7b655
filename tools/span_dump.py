"""DTGPU_DEBUG bit 4: the replay dumps its span list (document order) after command k instead of
the text.  python tools/span_dump.py git-makefile k out.txt"""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["DTGPU_DEBUG"] = str(16 + 256 * (int(sys.argv[2]) + 1))

import dt_amd
import golden_data as G

b = dt_amd.Batch(docs=[G.dt_bytes(sys.argv[1])], staging="host")
b.run()
b.sync()
raw = b.text(0)
vals = struct.unpack("<%dI" % (len(raw) // 4), raw)
with open(sys.argv[3], "w") as f:
    for i in range(0, len(vals), 2):
        w = vals[i + 1]
        f.write("%d %d %d\n" % (vals[i], w & 0xFFFFF, w >> 21))
print("spans", len(vals) // 2)
