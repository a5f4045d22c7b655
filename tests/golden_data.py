"""Loaders for the reference's own fixture files, copied verbatim into tests/golden/.

benchmark_data/* and causal_graph/*.json are data files from the reference repository
(/root/reference/benchmark_data, /root/reference/test_data/causal_graph).  The byte vectors
below are the `compat_*` known-answer vectors of src/list/encoding/tests.rs:374-424.
"""
import gzip
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
BENCH = os.path.join(HERE, "golden", "benchmark_data")
CG = os.path.join(HERE, "golden", "causal_graph")

DT_FILES = ["friendsforever", "git-makefile", "node_nodecc"]
JSON_TRACES = ["automerge-paper", "rustcode", "seph-blog1", "sveltecomponent", "friendsforever_flat"]


def dt_bytes(name):
    with open(os.path.join(BENCH, name + ".dt"), "rb") as f:
        return f.read()


_trace_cache = {}


def trace(name):
    if name not in _trace_cache:
        with gzip.open(os.path.join(BENCH, name + ".json.gz")) as f:
            _trace_cache[name] = json.load(f)
    return _trace_cache[name]


def cg_fixture(name):
    with open(os.path.join(CG, name + ".json")) as f:
        return [json.loads(l) for l in f if l.strip()]


# src/list/encoding/tests.rs:374-391 (compat_empty_doc)
COMPAT_EMPTY_1 = bytes([0x44, 0x4d, 0x4e, 0x44, 0x54, 0x59, 0x50, 0x53, 0x00, 0x01, 0x02, 0x03, 0x00, 0x0a, 0x07, 0x0c,
                        0x02, 0x00, 0x00, 0x0d, 0x01, 0x04, 0x14, 0x06, 0x15, 0x00, 0x16, 0x00, 0x17, 0x00, 0x64, 0x04,
                        0x6c, 0xce, 0x6b, 0x00])
COMPAT_EMPTY_2 = bytes([0x44, 0x4d, 0x4e, 0x44, 0x54, 0x59, 0x50, 0x53, 0x00, 0x01, 0x02, 0x03, 0x00, 0x0a, 0x00, 0x14,
                        0x06, 0x15, 0x00, 0x16, 0x00, 0x17, 0x00, 0x64, 0x04, 0x86, 0x77, 0x4d, 0x6a])
# src/list/encoding/tests.rs:393-424 (compat_simple_doc): "hi there", delete 3..7, insert "m"@3
COMPAT_SIMPLE_1 = bytes([68, 77, 78, 68, 84, 89, 80, 83, 0, 1, 7, 3, 5, 4, 115, 101, 112, 104, 10, 7, 12, 2, 0, 0, 13, 1, 4,
                         20, 32, 24, 16, 0, 13, 10, 4, 104, 105, 32, 116, 104, 101, 114, 101, 109, 25, 1, 19, 21, 2, 2,
                         13, 22, 4, 65, 79, 11, 0, 23, 2, 13, 1, 100, 4, 162, 205, 138, 38])
COMPAT_SIMPLE_2 = bytes([68, 77, 78, 68, 84, 89, 80, 83, 0, 1, 7, 3, 5, 4, 115, 101, 112, 104, 10, 0, 20, 32, 24, 16, 0, 13,
                         10, 4, 104, 105, 32, 116, 104, 101, 114, 101, 109, 25, 1, 19, 21, 2, 2, 13, 22, 4, 65, 79, 11, 0,
                         23, 2, 13, 1, 100, 4, 151, 117, 95, 151])
COMPAT_SIMPLE_LZ4 = bytes([68, 77, 78, 68, 84, 89, 80, 83, 0, 5, 11, 9, 144, 104, 105, 32, 116, 104, 101, 114, 101, 109, 1,
                           7, 3, 5, 4, 115, 101, 112, 104, 10, 0, 20, 24, 24, 8, 0, 14, 2, 4, 9, 25, 1, 19, 21, 2, 2, 13,
                           22, 4, 65, 79, 11, 0, 23, 2, 13, 1, 100, 4, 128, 32, 8, 191])
COMPAT_SIMPLE_TEXT = "hi me"
