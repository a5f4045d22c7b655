"""Extract the byte-vector fixtures held in the reference's encoding tests into JSON data.

Run in the build container (needs /root/reference); the output decode_vectors.json is committed
so the GPU box never reads the reference.  Source: src/list/encoding/tests.rs
(`merge_when_parents_unsorted`, `regression_1`).
"""
import json
import os
import re

SRC = "/root/reference/src/list/encoding/tests.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "decode_vectors.json")


def main():
    text = open(SRC).read()
    out = {}
    for test in ("merge_when_parents_unsorted", "regression_1"):
        i = text.index("fn " + test)
        j = text.index("\n}\n", i)
        body = text[i:j]
        for m in re.finditer(r"^\s*let (\w+): Vec<u8> = vec!\[([0-9, ]+)\];", body, re.M):
            out[f"{test}.{m.group(1)}"] = [int(x) for x in m.group(2).split(",") if x.strip()]
    with open(OUT, "w") as f:
        json.dump(out, f)
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
