"""Build record of libdtgpu (written by diamond-types_amd/Makefile after every link): the compiler,
the target, the flags, and a SHA-256 of every source and header the library is built from.
dt_amd.lib() compares the recorded hashes with the sources next to it and refuses a library built
from other sources (a stale prebuilt binary shipped with edited sources).
Usage: python3 tools/build_info.py OUT.json LIB.so -- FLAG... -- SOURCE..."""
import hashlib
import json
import os
import subprocess
import sys


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    out, lib = sys.argv[1], sys.argv[2]
    rest = sys.argv[3:]
    i = rest.index("--", 1)
    flags, srcs = rest[1:i], rest[i + 1:]
    base = os.path.dirname(os.path.abspath(lib))
    try:
        cc = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True, text=True).stdout.splitlines()
    except OSError:
        cc = []
    rec = {
        "build_mode": "release (make -C diamond-types_amd; __graft_entry__.build())",
        "compiler": [l for l in cc if l.strip()][:2],
        "flags": flags,
        "library": {"file": os.path.basename(lib), "sha256": sha(lib)},
        "sources": {os.path.relpath(os.path.abspath(s), os.path.dirname(base)): sha(s) for s in sorted(srcs)},
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
