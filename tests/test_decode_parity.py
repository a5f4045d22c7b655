"""Decode parity against the independent oracle, element by element.

The host decoder (dt_host.cpp::decode_dt) and the oracle (oracle/dt_oracle.c decode_internal)
both restate src/list/encoding/decode_oplog.rs; here every array the product exports --
op runs (expanded per LV with the reference's positional semantics, op_metrics.rs:184-202),
agent runs, graph entries and parents, per-LV content byte offsets, content, version and agent
names -- is compared with the oracle's.  tests/test_gpu_decode.py compares the device decoder
with the host decoder array by array, so the device decode chains to the oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, ROOT)
import dt_amd  # noqa: E402
import golden_data as G  # noqa: E402
from oracle.oracle import OpLog as OracleOpLog  # noqa: E402

NONE32 = 0xFFFFFFFF


def per_lv(ops):
    """Host op runs -> per-LV (kind, position): an insert run types forward (char i at pos + i)
    or is a reversed run (every char at pos); a delete run deletes at pos (forward) or, as a
    backspace run of span [pos, pos + len), at pos + len - 1 - i (op_metrics.rs:184-202)."""
    out = []
    for lv, ln, pos, kf in ops:
        kind, fwd = kf & 1, (kf >> 1) & 1
        for i in range(ln):
            if kind == 0:
                out.append((0, pos + i if fwd else pos))
            else:
                out.append((1, pos if fwd else pos + ln - 1 - i))
    return out


def compare(data):
    h = dt_amd.ListOpLog.load_from(data)
    o = OracleOpLog.load_from(data).decoded()
    ops = [tuple(r) for r in h.export("ops")]
    assert [r[0] for r in ops] == sorted(r[0] for r in ops)
    lvs = per_lv(ops)
    assert len(lvs) == len(o["lv"]) == len(h)
    assert lvs == [(k, p) for k, p, _ in o["lv"]]
    co = list(h.export("char_offsets"))
    assert [c if c != NONE32 else -1 for c in co] == [c for _, _, c in o["lv"]]
    assert [tuple(r) for r in h.export("agent_runs")] == [tuple(r) for r in o["agent_runs"]]
    ents = [tuple(e) for e in h.export("entries")]
    offs = list(h.export("parent_offsets"))
    pars = list(h.export("parents"))
    got = [(s, e, tuple(pars[offs[i]:offs[i + 1]])) for i, (s, e) in enumerate(ents)]
    assert got == o["entries"]
    assert list(h.export("version")) == o["version"]
    assert [n.decode() if isinstance(n, bytes) else n for n in h.export("agent_names")] == o["agent_names"]
    assert bytes(h.export("content")) == o["content"]


@pytest.mark.parametrize("name", G.DT_FILES)
def test_host_decoder_equals_oracle_arrays(name):
    compare(G.dt_bytes(name))


@pytest.mark.parametrize("vec", [G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_LZ4])
def test_host_decoder_equals_oracle_arrays_compat(vec):
    compare(vec)


@pytest.mark.parametrize("doc", [0, 1, 7, 42])
def test_host_decoder_equals_oracle_arrays_synthetic(doc):
    compare(dt_amd.synth_oplog(doc, 3000).encode())
