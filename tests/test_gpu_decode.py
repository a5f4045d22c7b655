"""GPU `.dt` decode (dt_decode.hip) vs the host decoder and the C oracle.

The device decoder must reproduce `ListOpLog::load_from` (src/list/encoding/decode_oplog.rs:447-960)
exactly: every decoded array equal to the host decoder's (which test_host_cpu.py pins to the
oracle), and on corrupted input the same `ParseError` code as the oracle.  A document may be
handed back to the host (DECODE_DEFER) only for the documented limits; no fixture here is.
"""
import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, OracleError

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402

WHAT = ["ops", "agent_runs", "entries", "parent_offsets", "parents", "content", "char_offsets", "version",
        "agent_names"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _host_code(data, ignore_crc=False):
    try:
        dt_amd.ListOpLog.load_from(data, ignore_crc=ignore_crc)
        return 0
    except dt_amd.ParseError as e:
        return e.code


def _oracle_code(data):
    try:
        OracleOpLog.load_from(data)
        return 0
    except OracleError as e:
        return e.code


def _same_arrays(dec, i, data, ignore_crc=False):
    host = dt_amd.ListOpLog.load_from(data, ignore_crc=ignore_crc)
    for w in WHAT:
        a, b = dec.export(i, w), host.export(w)
        if w == "agent_names":
            assert a == b, w
        else:
            assert np.array_equal(a, b), (w, a[:8], b[:8])
    st = dec.status(i)
    assert st["n_lv"] == len(host)


@pytest.mark.parametrize("name", G.DT_FILES)
def test_benchmark_files_decode_identically(name):
    data = G.dt_bytes(name)
    dec = dt_amd.DecodeBatch([data])
    dec.run()
    assert dec.status(0)["status"] == 0
    _same_arrays(dec, 0, data)


def test_compat_vectors_decode_identically():
    docs = [G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_LZ4, G.COMPAT_EMPTY_1, G.COMPAT_EMPTY_2]
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        _same_arrays(dec, i, d)


def test_mixed_batch_and_repeat_runs():
    docs = [G.dt_bytes(n) for n in G.DT_FILES] * 3 + [G.COMPAT_SIMPLE_LZ4, b"", b"DMNDTYPS"]
    dec = dt_amd.DecodeBatch(docs)
    for _ in range(2):
        dec.run()
        for i, d in enumerate(docs):
            want = _host_code(d)
            assert dec.status(i)["status"] == want, i
            if want == 0:
                _same_arrays(dec, i, d)


@pytest.mark.parametrize("vec", ["COMPAT_SIMPLE_LZ4", "COMPAT_SIMPLE_1"])
def test_parse_error_codes_on_every_corruption(vec):
    """Every single-byte corruption and every truncation: device status == oracle ParseError."""
    base = bytearray(getattr(G, vec))
    docs = []
    for i in range(len(base)):
        for flip in (0xFF, 0x01, 0x80, 0x7F):
            b = bytearray(base)
            b[i] ^= flip
            docs.append(bytes(b))
    docs += [bytes(base[:cut]) for cut in range(len(base))]
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    deferred = 0
    for i, d in enumerate(docs):
        got = dec.status(i)["status"]
        if got == dt_amd.DECODE_DEFER:
            deferred += 1
            continue
        assert got == _oracle_code(d) == _host_code(d), (i, d.hex())
        if got == 0:
            _same_arrays(dec, i, d)
    assert deferred <= len(docs) // 20


def test_corrupted_benchmark_file():
    data = bytearray(G.dt_bytes("friendsforever"))
    rng = np.random.default_rng(7)
    docs = []
    for _ in range(48):
        b = bytearray(data)
        b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
        docs.append(bytes(b))
    for cut in (9, 20, 100, 1000, len(data) // 2, len(data) - 5):
        docs.append(bytes(data[:cut]))
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        got = dec.status(i)["status"]
        if got == dt_amd.DECODE_DEFER:
            continue
        assert got == _host_code(d), i
    # the same bytes with the CRC check disabled decode like the host decoder does
    dec2 = dt_amd.DecodeBatch(docs[:16], ignore_crc=True)
    dec2.run()
    for i, d in enumerate(docs[:16]):
        got = dec2.status(i)["status"]
        if got != dt_amd.DECODE_DEFER:
            assert got == _host_code(d, ignore_crc=True), i
            if got == 0:
                _same_arrays(dec2, i, d, ignore_crc=True)


@pytest.mark.parametrize("name", G.DT_FILES)
def test_fast_path_taken_on_benchmark_files(name):
    """The benchmark files are the plain case (ASCII inserts in known runs, no delete content):
    the lane-parallel fast path must decode them itself.  Its agent-assignment half leaves a
    nonzero cycle count in profile slot 7; when it bails the exact path still yields the same
    arrays, so only this check notices a fast path that silently stopped working."""
    data = G.dt_bytes(name)
    dec = dt_amd.DecodeBatch([data])
    dec.run()
    assert dec.status(0)["status"] == 0
    assert dec.profile(0)[7] > 0


def _lz4_shape_docs():
    """Documents whose LZ4-compressed insert content covers the decompressor's cases: runs with
    match offsets 1-3 (overlapping, periodic copies) and length-extension chains past 255, long
    literal runs (extension bytes, 255 chains), matches reaching back more than one 64-sequence
    batch and more than one 256-byte window, and short texts that stay uncompressed; with blocks
    past 64 KB in the batch, the copy's resolved-source ring is on."""
    import random
    rng = random.Random(7)
    vocab = ["".join(rng.choice("abcdefghij ") for _ in range(rng.randint(2, 9))) for _ in range(40)]
    texts = [
        "a" * 1000,
        "ab" * 300 + "xyz" * 200,
        "".join(chr(33 + rng.randrange(90)) for _ in range(300)),
        "".join(chr(33 + rng.randrange(90)) for _ in range(5000)),
        " ".join(rng.choice(vocab) for _ in range(20000)),
        "q" * 20 + "".join(chr(33 + rng.randrange(90)) for _ in range(17)) + "q" * 300,
        "short",
        # blocks past 64 KB (the batch then runs the copy's resolved-source ring): one run longer
        # than a 4 KB mapped batch, a period of 37 across rounds, matches reaching past the ring
        "a" * 70000,
        "0123456789abcdefghijklmnopqrstuvwxyz!" * 3000,
        "".join(chr(33 + rng.randrange(90)) for _ in range(3000)) * 25,
    ]
    docs = []
    for t in texts:
        o = dt_amd.ListOpLog()
        a = o.get_or_create_agent_id("lz")
        pos = 0
        for i in range(0, len(t), 997):   # several insert runs
            piece = t[i:i + 997]
            o.add_insert(a, pos, piece)
            pos += len(piece)
        docs.append(o.encode(dt_amd.ENCODE_FULL))
    return docs


def test_lz4_shapes_decode_identically():
    docs = _lz4_shape_docs()
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        _same_arrays(dec, i, d)


def test_lz4_shapes_single_wave(monkeypatch):
    """The same documents with the two-wave LZ4 kernel off (DTGPU_NO_LZ_PRE): every block is
    decompressed inside decode_kernel by one wave."""
    monkeypatch.setenv("DTGPU_NO_LZ_PRE", "1")
    docs = _lz4_shape_docs()
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        _same_arrays(dec, i, d)


@pytest.mark.parametrize("lz3_max", ["4096", "0"])
def test_lz4_many_long_blocks(monkeypatch, lz3_max):
    """540 documents with a long LZ4 block, on the three-wave kernel (up to 4,096 blocks) and on
    the two-wave one (DTGPU_LZ3_MAX=0, as past that): every copy decodes like the host decoder."""
    monkeypatch.setenv("DTGPU_LZ3_MAX", lz3_max)
    shapes = _lz4_shape_docs()[-3:]
    docs = [shapes[i % 3] for i in range(540)]
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
    for i in (0, 1, 2, 271, 539):
        _same_arrays(dec, i, docs[i])


def test_long_documents_uncompressed():
    """Documents past the deferred-fill threshold (131,072 LVs) written without LZ4: fill_kernel
    copies their insert text from the document bytes instead of the LZ4 buffer (and their per-LV
    offsets, ASCII and non-ASCII, from the deferred jobs)."""
    opts = dt_amd.EncodeOptions(True, False, True)
    docs = [dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode(opts) for n in ("automerge-paper", "rustcode")]
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        _same_arrays(dec, i, d)


def test_lz4_corrupt_long_blocks():
    """Corruptions of documents whose LZ4 block goes through the two-wave kernel: the verdict
    (status and, when it decodes, the arrays) equals the host decoder's."""
    import random
    rng = random.Random(11)
    base = _lz4_shape_docs()[-3:]
    docs = []
    for d in base:
        for _ in range(6):
            b = bytearray(d)
            for _ in range(rng.randint(1, 4)):
                k = rng.randrange(16, len(b))
                b[k] = rng.randrange(256)
            docs.append(bytes(b))
    for crc in (False, True):   # with the CRC check off, the LZ4 verdicts themselves are compared
        dec = dt_amd.DecodeBatch(docs, ignore_crc=not crc)
        dec.run()
        for i, d in enumerate(docs):
            got = dec.status(i)["status"]
            if got == dt_amd.DECODE_DEFER:
                continue
            want = _host_code(d, ignore_crc=not crc)
            assert got == want, (crc, i, got, want)
            if want == 0:
                _same_arrays(dec, i, d, ignore_crc=not crc)


def _utf8_docs():
    """Non-ASCII insert text: the JSON traces whose content is not all ASCII, written as .dt the
    way configs[4] writes them, and small documents with 2-, 3- and 4-byte chars between ASCII
    ones, deletes and concurrent inserts."""
    docs = []
    for n in ("seph-blog1", "rustcode"):
        docs.append(dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode())
    o = dt_amd.ListOpLog()
    a, b = o.get_or_create_agent_id("a"), o.get_or_create_agent_id("b")
    o.add_insert(a, 0, "héllo wörld — ✓ 😀 end")
    o.add_delete_without_content(a, 3, 6)
    o.add_insert(b, 2, "ßü€𝄞")
    v = list(o.local_frontier())
    o.add_insert_at(a, v, 1, "日本語")
    o.add_insert_at(b, v, 4, "x😀y")
    o.add_insert(a, 0, "plain ascii at the front ")
    docs.append(o.encode())
    # continuation-byte counts around the 64 a register table holds (more take the char-numbering
    # pass), and multi-byte chars straddling the table pass's 1 KB strides
    for text in ("é" * 64, "é" * 65, "日本語テキスト" * 10, "a" * 1021 + "€" + "b" * 500 + "😀" + "c" * 2000):
        o = dt_amd.ListOpLog()
        a = o.get_or_create_agent_id("a")
        o.add_insert(a, 0, text)
        o.add_delete_without_content(a, 5, 3)
        o.add_insert(a, 7, "ü")
        docs.append(o.encode())
    return docs


def test_utf8_text_takes_the_batched_path():
    """Non-ASCII insert text decodes on the batched op-record path too (the char numbering, then
    each char's byte offset placed from the text): arrays equal the host decoder's, and profile
    slot 7 shows the batched path ran."""
    docs = _utf8_docs()
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        _same_arrays(dec, i, d)
        assert dec.profile(i)[7] > 0, i
