"""CPU-side tests of libdtgpu's host code and C ABI (no GPU needed): the library loads and
exports every symbol in include/dtgpu.h, the `.dt` decoder agrees with the oracle, ParseError
codes match, the planner's walk matches the oracle's, and checkout refuses to run without a
device (no CPU fallback)."""
import ctypes
import os
import re

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, OracleError, oplog_from_trace as oracle_from_trace
import dt_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "dtgpu.h")).read()
    names = set(re.findall(r"\b(dtgpu_[a-z0-9_]+)\s*\(", hdr))
    assert len(names) >= 25
    L = ctypes.CDLL(dt_amd.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert missing == []


@pytest.mark.parametrize("name", G.DT_FILES)
def test_decode_matches_oracle(name):
    data = G.dt_bytes(name)
    g = dt_amd.ListOpLog.load_from(data)
    o = OracleOpLog.load_from(data)
    assert len(g) == len(o)
    assert g.local_frontier() == o.frontier()


@pytest.mark.parametrize("name", G.DT_FILES)
def test_plan_matches_oracle_walk(name):
    data = G.dt_bytes(name)
    ps = dt_amd.ListOpLog.load_from(data).plan_stats()
    _, st = OracleOpLog.load_from(data).checkout_tip_bytes(order=0, with_stats=True)
    assert (ps["steps"], ps["retreat"], ps["advance"]) == (st["n_steps"], st["n_retreat"], st["n_advance"])


@pytest.mark.parametrize("vec", [G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_LZ4, G.COMPAT_EMPTY_1, G.COMPAT_EMPTY_2])
def test_compat_decode(vec):
    g = dt_amd.ListOpLog.load_from(vec)
    o = OracleOpLog.load_from(vec)
    assert (len(g), g.local_frontier()) == (len(o), o.frontier())


def _code(fn, data):
    try:
        fn(data)
        return 0
    except dt_amd.ParseError as e:
        return e.code
    except OracleError as e:
        return e.code


def test_parse_error_codes_match_oracle_on_corruption():
    base = bytearray(G.COMPAT_SIMPLE_LZ4)
    for i in range(len(base)):
        for flip in (0xFF, 0x01, 0x80, 0x7F, 0x40, 0x02):
            b = bytearray(base)
            b[i] ^= flip
            d = bytes(b)
            assert _code(dt_amd.ListOpLog.load_from, d) == _code(OracleOpLog.load_from, d), (i, flip)
    for cut in range(len(base)):
        d = bytes(base[:cut])
        assert _code(dt_amd.ListOpLog.load_from, d) == _code(OracleOpLog.load_from, d), cut


def test_ignore_crc():
    b = bytearray(G.COMPAT_SIMPLE_1)
    b[-1] ^= 0xFF
    with pytest.raises(dt_amd.ParseError) as e:
        dt_amd.ListOpLog.load_from(bytes(b))
    assert e.value.name == "ChecksumFailed"
    assert len(dt_amd.ListOpLog.load_from(bytes(b), ignore_crc=True)) == 13


def test_builder_api_matches_oracle():
    g = dt_amd.ListOpLog()
    o = OracleOpLog()
    a1, a2 = g.get_or_create_agent_id("a"), o.agent("a")
    b1, b2 = g.get_or_create_agent_id("b"), o.agent("b")
    assert (a1, b1) == (a2, b2) == (0, 1)
    assert g.add_insert_at(a1, [], 0, "aaa") == o.add_insert_at(a2, [], 0, "aaa") == 2
    assert g.add_insert_at(b1, [], 0, "bbb") == o.add_insert_at(b2, [], 0, "bbb") == 5
    assert g.local_frontier() == o.frontier() == [2, 5]
    assert g.add_insert_at(a1, [2, 5], 0, "ccc") == 8
    assert g.local_frontier() == [8]
    with pytest.raises(ValueError):
        g.get_or_create_agent_id("ROOT")


def test_trace_builder_matches_oracle():
    t = G.trace("friendsforever_flat")
    g = dt_amd.oplog_from_trace(t["txns"])
    o = oracle_from_trace(t["txns"])
    assert len(g) == len(o) and g.local_frontier() == o.frontier()
    ps = g.plan_stats()
    assert ps["steps"] == 1 and ps["retreat"] == 0


def test_text_hash_definition():
    import struct
    data = "héllo".encode()
    h = 0
    for i, byte in enumerate(data):
        z = ((i << 8) | byte) + 0x9E3779B97F4A7C15 & (2**64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        h = (h + (z ^ (z >> 31))) & (2**64 - 1)
    assert dt_amd.text_hash(data) == h


def test_no_cpu_fallback_without_device():
    if dt_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(dt_amd.ParseError) as e:
        dt_amd.ListOpLog.load_from(G.COMPAT_SIMPLE_1).checkout_tip()
    assert e.value.name == "ErrNoDevice"
