"""`.dt` encoder: `ListOpLog::encode` / `encode_from` (src/list/encoding/encode_oplog.rs:404-747),
libdtgpu's dtgpu_oplog_encode (host code, csrc/dt_encode.cpp).

LZ4 (lz4_flex 0.10's block compressor, encode_oplog.rs:320-343): the LZ4 blocks the reference
wrote into friendsforever.dt, git-makefile.dt and node_nodecc.dt are reproduced byte for byte from
their decompressed content (decompressed by the oracle), covering both hash tables (inputs below
and above 64 KiB), and compat_simple_doc's LZ4 vector (tests.rs:404-415) too.

Byte-exact against the reference encoder's own outputs held in its tests
(src/list/encoding/tests.rs): `compat_simple_doc` bytes2 (:418) and `compat_empty_doc` bytes2
(:383) exactly; `regression_1` doc_data (:362) exactly up to the older StartBranch-at-ROOT form
that file carries (tests.rs:379-383 documents that change).  Semantically on the benchmark files
and the other vectors: the re-decoded oplog holds the same ops, keyed by (agent, seq), with the
same parents, and checks out to the same text.
"""
import ctypes
import json
import os
import struct

import pytest

import golden_data as G
from dt_encode import crc32c
from oracle.oracle import OpLog as OracleOpLog
import dt_amd
from oracle import oracle as O


def _leb(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return v, i


def _lz4_chunk(data):
    """The leading CompressedFieldsLZ4 chunk of a `.dt` file: (uncompressed length, raw block)."""
    assert data[:8] == b"DMNDTYPS"
    _, i = _leb(data, 8)
    t, i = _leb(data, i)
    n, i = _leb(data, i)
    assert t == 5
    ul, j = _leb(data[i:i + n], 0)
    return ul, data[i + j:i + n]


def _oracle_lz4_decompress(block, ul):
    out = ctypes.create_string_buffer(max(1, ul))
    assert O.lib().dto_lz4_decompress(block, len(block), out, ul) == 0
    return out.raw[:ul]

VECTORS = json.load(open(os.path.join(G.HERE, "golden", "decode_vectors.json")))
OLD_START_BRANCH = bytes([10, 7, 12, 2, 0, 0, 13, 1, 4])   # StartBranch{Version[ROOT], Content ""}


def _keyed(o):
    """Per op, keyed by (agent name, seq): (kind, position, char, parents as (agent, seq))."""
    names = o.export("agent_names")
    names = [n.decode() if isinstance(n, bytes) else n for n in names]
    av = {}
    for lv, ln, agent, seq in o.export("agent_runs").reshape(-1, 4):
        for k in range(int(ln)):
            av[int(lv) + k] = (names[int(agent)], int(seq) + k)
    ents = o.export("entries").reshape(-1, 2)
    off = o.export("parent_offsets")
    par = o.export("parents")
    starts = {int(s): [av[int(p)] for p in par[off[i]:off[i + 1]]] for i, (s, _e) in enumerate(ents)}
    content = bytes(o.export("content"))
    coff = o.export("char_offsets")
    out = {}
    for lv, ln, pos, kf in o.export("ops").reshape(-1, 4):
        lv, ln, pos, kf = int(lv), int(ln), int(pos), int(kf)
        for k in range(ln):
            v = lv + k
            if kf & 1 == 0:
                b = int(coff[v])
                at, ch = pos + k, content[b:b + 4].decode("utf-8", errors="ignore")[:1]
            else:
                at, ch = (pos if kf & 2 else pos + ln - 1 - k), None
            ps = starts.get(v, [av[v - 1]] if v else [])
            out[av[v]] = (kf & 1, at, ch, tuple(sorted(ps)))
    return out


def test_compat_vectors_byte_exact():
    assert dt_amd.ListOpLog.load_from(G.COMPAT_SIMPLE_2).encode() == bytes(G.COMPAT_SIMPLE_2)
    assert dt_amd.ListOpLog.load_from(G.COMPAT_EMPTY_2).encode() == bytes(G.COMPAT_EMPTY_2)
    assert dt_amd.ListOpLog().encode() == bytes(G.COMPAT_EMPTY_2)
    # the older encodings of the same documents decode to the same oplog, which encodes to bytes2
    for v in (G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_LZ4):
        assert dt_amd.ListOpLog.load_from(v).encode() == bytes(G.COMPAT_SIMPLE_2)
    assert dt_amd.ListOpLog.load_from(G.COMPAT_EMPTY_1).encode() == bytes(G.COMPAT_EMPTY_2)


def test_builder_doc_matches_compat_simple():
    """compat_simple_doc's construction (tests.rs:396-400) encodes to the reference's bytes2."""
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("seph")
    o.add_insert(a, 0, "hi there")
    o.add_delete_without_content(a, 3, 7)
    o.add_insert(a, 3, "m")
    assert o.encode() == bytes(G.COMPAT_SIMPLE_2)


def test_regression_1_doc_byte_exact_up_to_start_branch_form():
    v = bytes(VECTORS["regression_1.doc_data"])
    e = dt_amd.ListOpLog.load_from(v).encode()
    i = e.index(bytes([10, 0, 20]))
    old = e[:i] + OLD_START_BRANCH + e[i + 2:-6]
    assert old + bytes([100, 4]) + struct.pack("<I", crc32c(old)) == v


@pytest.mark.parametrize("name", G.DT_FILES)
def test_benchmark_files_round_trip(name):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    e = o.encode()
    back = dt_amd.ListOpLog.load_from(e)
    assert len(back) == len(o)
    assert _keyed(back) == _keyed(o)
    if name != "node_nodecc":
        assert OracleOpLog.load_from(e).checkout_tip_bytes() == OracleOpLog.load_from(data).checkout_tip_bytes()


@pytest.mark.parametrize("key", sorted(VECTORS))
def test_vectors_round_trip(key):
    o = dt_amd.ListOpLog.load_from(bytes(VECTORS[key]), ignore_crc=False) if key != "regression_1.patch_data" else None
    if o is None:
        pytest.skip("a patch: decodes only on top of its base document (decode_and_add)")
    back = dt_amd.ListOpLog.load_from(o.encode())
    assert _keyed(back) == _keyed(o)


def test_synthetic_round_trip():
    for doc in range(3):
        o = dt_amd.synth_oplog(doc, 2000)
        back = dt_amd.ListOpLog.load_from(o.encode())
        assert _keyed(back) == _keyed(o)


def test_encode_from_version_holds_only_the_new_ops():
    o = dt_amd.ListOpLog.load_from(G.dt_bytes("friendsforever"))
    v = [12000]
    patch = o.encode_from(v, dt_amd.ENCODE_PATCH)
    assert len(patch) < len(o.encode())
    with pytest.raises(Exception):
        dt_amd.ListOpLog.load_from(patch)   # foreign parents: BaseVersionUnknown on an empty oplog


@pytest.mark.parametrize("name", G.DT_FILES)
def test_lz4_compressor_reproduces_the_reference_blocks(name):
    ul, block = _lz4_chunk(G.dt_bytes(name))
    raw = _oracle_lz4_decompress(block, ul)
    assert dt_amd.lz4_compress(raw) == block


def test_lz4_compat_vector_and_short_inputs():
    ul, block = _lz4_chunk(bytes(G.COMPAT_SIMPLE_LZ4))
    assert dt_amd.lz4_compress(_oracle_lz4_decompress(block, ul)) == block
    for n in (0, 1, 12, 13, 20, 100):   # literal-only below 13 bytes; every block decodes back
        data = bytes((i * 7) % 5 + 97 for i in range(n))
        c = dt_amd.lz4_compress(data)
        assert _oracle_lz4_decompress(c, n) == data
        if n < 13:
            assert c[0] >> 4 == min(n, 15) and len(c) == 1 + n + (n >= 15)


def test_encode_full_compresses_content_of_20_bytes_or_more():
    """write_content (encode_oplog.rs:270-305): content >= 20 bytes goes into the leading LZ4
    chunk as ContentCompressed; shorter content stays inline; ENCODE_PATCH compresses too and
    compress_content = false writes Content."""
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("seph")
    o.add_insert(a, 0, "the quick brown fox jumps over the lazy dog " * 4)
    full = o.encode()
    assert full[9] == 5 and o.encode(dt_amd.ENCODE_PATCH) == full
    plain = o.encode(dt_amd.EncodeOptions(True, False, True))
    assert plain[9] != 5 and len(plain) > len(full)
    for data in (full, plain):
        assert OracleOpLog.load_from(data).checkout_tip_bytes() == b"the quick brown fox jumps over the lazy dog " * 4
        assert _keyed(dt_amd.ListOpLog.load_from(data)) == _keyed(o)
    short = dt_amd.ListOpLog()
    short.add_insert(short.get_or_create_agent_id("seph"), 0, "nineteen characters")
    assert short.encode()[9] != 5


@pytest.mark.parametrize("name", G.DT_FILES)
def test_benchmark_files_encode_full_compressed(name):
    """ENCODE_FULL of a benchmark file: one LZ4 chunk holding the inserted text in the encoder's
    walk order, which the oracle decompresses and decodes to the same history."""
    o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
    e = o.encode()
    ul, block = _lz4_chunk(e)
    raw = _oracle_lz4_decompress(block, ul)
    assert ul == len(bytes(o.export("content"))) and sorted(raw) == sorted(bytes(o.export("content")))
    assert dt_amd.lz4_compress(raw) == block
    assert len(OracleOpLog.load_from(e)) == len(o)
