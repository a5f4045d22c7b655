"""dt_amd -- Python mirror of diamond-types' `ListOpLog` / `ListBranch` checkout surface,
backed by libdtgpu (hand-written HIP kernels for MI355X, C ABI in include/dtgpu.h).

Mirrors (reference paths under jarrodhroberson/diamond-types):
  ListOpLog.load_from          src/list/encoding/decode_oplog.rs:447
  ListOpLog.checkout_tip       src/list/oplog.rs:38  (device replay: dt_replay.hip)
  ListOpLog.add_insert_at ...  src/list/oplog.rs:221-300
  ListBranch.content / len     src/list/branch.rs:38-63
  batch_checkout               SURVEY.md §8b batch entry

There is no CPU fallback: every checkout runs the HIP kernels, and a missing library or a
missing GPU raises immediately.
"""
import collections
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DTGPU_LIB_DIR: an alternative in-tree build (A/B experiments, e.g. lib_exp/); default lib/
LIB_PATH = os.path.join(os.path.dirname(_HERE), os.environ.get("DTGPU_LIB_DIR", "lib"), "libdtgpu.so")

STATUS_NAMES = {
    0: "OK", 1: "InvalidMagic", 2: "UnsupportedProtocolVersion", 3: "DocIdMismatch", 4: "BaseVersionUnknown",
    5: "UnknownChunk", 6: "LZ4DecoderNeeded", 7: "LZ4DecompressionError", 8: "CompressedDataMissing",
    9: "InvalidChunkHeader", 10: "MissingChunk", 11: "InvalidLength", 12: "UnexpectedEOF", 13: "InvalidUTF8",
    14: "InvalidRemoteID", 15: "InvalidVarInt", 16: "InvalidContent", 17: "GenericInvalidData",
    18: "ChecksumFailed", 19: "DataMissing", 64: "ErrCheckout", 65: "ErrCapacity", 66: "ErrHip", 67: "ErrArg",
    68: "ErrNoDevice",
}


class ParseError(Exception):
    """Mirror of `ParseError` (src/encoding/parseerror.rs:14-48) plus engine statuses."""

    def __init__(self, code):
        self.code = code
        self.name = STATUS_NAMES.get(code, str(code))
        super().__init__(f"{self.name} ({code})")


class DocResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("text_len", ctypes.c_uint64),
                ("text_hash", ctypes.c_uint64), ("n_lv", ctypes.c_uint64)]


class BatchOpts(ctypes.Structure):
    """dtgpu_batch_opts (include/dtgpu.h): flags = DTGPU_OPT_* (OPT_* below); seg_ops / seg_max /
    lds_fill 0 = defaults.  DTGPU_* environment variables override them at batch creation."""
    _fields_ = [("ignore_crc", ctypes.c_int), ("host_threads", ctypes.c_int), ("device", ctypes.c_int),
                ("flags", ctypes.c_uint32), ("seg_ops", ctypes.c_uint32), ("seg_max", ctypes.c_uint32),
                ("lds_fill", ctypes.c_uint32)]


OPT_NO_FAST_FORWARD, OPT_NO_SEGMENTS, OPT_HOST_PLAN, OPT_NO_SPLIT, OPT_NO_CRITICAL, OPT_DEBUG, OPT_PASS_MARK = \
    1, 2, 4, 8, 16, 32, 64


class GraphQuery(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("graph", ctypes.c_uint32), ("na", ctypes.c_size_t),
                ("nb", ctypes.c_size_t), ("a", ctypes.POINTER(ctypes.c_int64)), ("b", ctypes.POINTER(ctypes.c_int64)),
                ("target", ctypes.c_int64)]


class GraphAnswer(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("n_a", ctypes.c_uint32), ("n_b", ctypes.c_uint32),
                ("n_common", ctypes.c_uint32)]


_lib = None


def _check_build_record():
    """The library's build record (lib/build_info.json, tools/build_info.py) names the hash of every
    source it was built from: a library built from other sources than the ones beside it (a stale
    prebuilt binary) is refused.  Experiment builds without a record (DTGPU_LIB_DIR) load as they are."""
    import hashlib
    import json
    info = os.path.join(os.path.dirname(LIB_PATH), "build_info.json")
    if not os.path.exists(info):
        return
    with open(info) as f:
        rec = json.load(f)
    pkg = os.path.dirname(os.path.dirname(LIB_PATH))
    stale = []
    for rel, h in rec.get("sources", {}).items():
        path = os.path.join(pkg, rel)
        if os.path.exists(path):
            with open(path, "rb") as f:
                if hashlib.sha256(f.read()).hexdigest() != h:
                    stale.append(rel)
    if stale:
        raise RuntimeError(f"{LIB_PATH} was built from other sources than {', '.join(stale[:4])}"
                           f"{' ...' if len(stale) > 4 else ''}; rebuild with `make -C diamond-types_amd`")


def lib():
    """Load libdtgpu.so (fails loudly when it has not been built, or was built from other sources)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libdtgpu.so not built at {LIB_PATH}; run `make -C diamond-types_amd`")
    _check_build_record()
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u64, i64, c = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
    pu64 = ctypes.POINTER(ctypes.c_uint64)
    L.dtgpu_oplog_load.argtypes = [ctypes.c_char_p, sz, c, ctypes.POINTER(vp)]
    L.dtgpu_oplog_new.restype = vp
    L.dtgpu_oplog_free.argtypes = [vp]
    L.dtgpu_oplog_get_or_create_agent_id.argtypes = [vp, ctypes.c_char_p, sz]
    L.dtgpu_oplog_get_or_create_agent_id.restype = ctypes.c_int32
    L.dtgpu_oplog_add_insert_at.argtypes = [vp, ctypes.c_int32, pu64, sz, u64, ctypes.c_char_p, sz]
    L.dtgpu_oplog_add_insert_at.restype = i64
    L.dtgpu_oplog_add_delete_at.argtypes = [vp, ctypes.c_int32, pu64, sz, u64, u64]
    L.dtgpu_oplog_add_delete_at.restype = i64
    L.dtgpu_oplog_add_insert.argtypes = [vp, ctypes.c_int32, u64, ctypes.c_char_p, sz]
    L.dtgpu_oplog_add_insert.restype = i64
    L.dtgpu_oplog_add_delete_without_content.argtypes = [vp, ctypes.c_int32, u64, u64]
    L.dtgpu_oplog_add_delete_without_content.restype = i64
    L.dtgpu_oplog_len.argtypes = [vp]
    L.dtgpu_oplog_len.restype = sz
    L.dtgpu_oplog_local_frontier.argtypes = [vp, pu64, sz]
    L.dtgpu_oplog_local_frontier.restype = sz
    L.dtgpu_oplog_plan_stats.argtypes = [vp, pu64]
    L.dtgpu_oplog_plan_commands.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_oplog_plan_commands.restype = sz
    L.dtgpu_oplog_plan_tlist.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_oplog_plan_tlist.restype = sz
    L.dtgpu_batch_last_times.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_batch_host_planned.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8), sz]
    L.dtgpu_batch_host_planned.restype = sz
    L.dtgpu_batch_fast_forwarded.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8), sz]
    L.dtgpu_batch_fast_forwarded.restype = sz
    pu32 = ctypes.POINTER(ctypes.c_uint32)
    L.dtgpu_batch_plan.argtypes = [vp, sz, pu32, sz, pu32, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.dtgpu_oplog_ins_content.argtypes = [vp, ctypes.c_char_p, sz]
    L.dtgpu_oplog_ins_content.restype = sz
    L.dtgpu_oplog_char_offsets.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_oplog_char_offsets.restype = sz
    L.dtgpu_oplog_agent_runs.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_oplog_agent_runs.restype = sz
    L.dtgpu_checkout_tip.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.dtgpu_checkout.argtypes = [vp, pu64, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.dtgpu_oplog_dominators.argtypes = [vp, pu64, sz, pu64, sz, pu64, sz]
    L.dtgpu_oplog_dominators.restype = ctypes.c_int64
    L.dtgpu_oplog_history.argtypes = [vp, pu64, sz, ctypes.POINTER(vp)]
    L.dtgpu_oplog_project.argtypes = [vp, pu64, sz, ctypes.POINTER(vp)]
    L.dtgpu_oplog_project_version.argtypes = [vp, pu64, sz, pu64, sz, pu64, sz]
    L.dtgpu_oplog_project_version.restype = i64
    L.dtgpu_oplog_local_to_remote.argtypes = [vp, u64, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(u64)]
    L.dtgpu_oplog_remote_to_local.argtypes = [vp, ctypes.c_uint32, u64, u64, pu64, sz]
    L.dtgpu_oplog_remote_to_local.restype = i64
    L.dtgpu_oplog_encode.argtypes = [vp, pu64, sz, ctypes.c_uint32, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.dtgpu_lz4_compress.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.dtgpu_oplog_decode_and_add.argtypes = [vp, ctypes.c_char_p, sz, c, pu64, sz, ctypes.POINTER(sz)]
    L.dtgpu_oplog_last_added_frontier.argtypes = [vp, pu64, sz]
    L.dtgpu_oplog_last_added_frontier.restype = sz
    L.dtgpu_oplog_doc_id.argtypes = [vp, ctypes.c_char_p, sz]
    L.dtgpu_oplog_doc_id.restype = ctypes.c_int64
    L.dtgpu_oplog_set_doc_id.argtypes = [vp, ctypes.c_char_p, sz]
    L.dtgpu_xf_operations.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz, ctypes.POINTER(sz)]
    L.dtgpu_oplog_xf_order.argtypes = [vp, pu64, sz, pu64, sz, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_oplog_xf_order.restype = sz
    L.dtgpu_xf_operations_from.argtypes = [vp, pu64, sz, pu64, sz, ctypes.POINTER(ctypes.c_uint32), sz,
                                           ctypes.POINTER(sz)]
    L.dtgpu_batch_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz,
                                     ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.dtgpu_batch_create_from_oplogs.argtypes = [ctypes.POINTER(vp), sz, ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.dtgpu_batch_create_xf.argtypes = [ctypes.POINTER(vp), sz, ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.dtgpu_batch_xf_positions.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32), sz, ctypes.POINTER(sz)]
    L.dtgpu_batch_run.argtypes = [vp, vp]
    L.dtgpu_batch_run_timed.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_batch_sync.argtypes = [vp]
    L.dtgpu_batch_size.argtypes = [vp]
    L.dtgpu_batch_size.restype = sz
    L.dtgpu_batch_results.argtypes = [vp, ctypes.POINTER(DocResult)]
    L.dtgpu_batch_text.argtypes = [vp, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.dtgpu_batch_algorithmic_bytes.argtypes = [vp]
    L.dtgpu_batch_algorithmic_bytes.restype = u64
    L.dtgpu_batch_doc_stats.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32)]
    L.dtgpu_batch_segments.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_batch_segments.restype = sz
    L.dtgpu_oplog_cut_ranges.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), sz]
    L.dtgpu_oplog_cut_ranges.restype = sz
    L.dtgpu_batch_plan_profile.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint64)]
    L.dtgpu_batch_total_lv.argtypes = [vp]
    L.dtgpu_batch_total_lv.restype = u64
    L.dtgpu_batch_free.argtypes = [vp]
    L.dtgpu_batch_create_device.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz,
                                            ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.dtgpu_batch_run_e2e_timed.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_batch_encode.argtypes = [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_batch_encoded.argtypes = [vp, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz), ctypes.POINTER(ctypes.c_uint64)]
    L.dtgpu_batch_encoded_bytes.argtypes = [vp, ctypes.c_int]
    L.dtgpu_batch_encoded_bytes.restype = ctypes.c_uint64
    L.dtgpu_batch_checkout.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz,
                                       ctypes.POINTER(BatchOpts), ctypes.POINTER(DocResult)]
    L.dtgpu_text_hash.argtypes = [ctypes.c_char_p, sz]
    L.dtgpu_text_hash.restype = u64
    L.dtgpu_device_count.restype = c
    L.dtgpu_synth_ops.argtypes = [u64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), sz]
    L.dtgpu_synth_ops.restype = sz
    L.dtgpu_synth_oplog.argtypes = [u64, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.dtgpu_synth_merge_oplog.argtypes = [u64, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(vp)]
    L.dtgpu_oplog_export.argtypes = [vp, c, vp, sz]
    L.dtgpu_oplog_export.restype = sz
    L.dtgpu_decode_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz,
                                      ctypes.POINTER(BatchOpts), ctypes.POINTER(vp)]
    L.dtgpu_decode_run.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_decode_size.argtypes = [vp]
    L.dtgpu_decode_size.restype = sz
    L.dtgpu_decode_status.argtypes = [vp, sz, pu64]
    L.dtgpu_decode_export.argtypes = [vp, sz, c, vp, sz]
    L.dtgpu_decode_export.restype = sz
    L.dtgpu_decode_bytes.argtypes = [vp, c]
    L.dtgpu_decode_bytes.restype = u64
    L.dtgpu_decode_last_ms.argtypes = [vp]
    L.dtgpu_decode_last_ms.restype = ctypes.c_float
    L.dtgpu_decode_free.argtypes = [vp]
    L.dtgpu_decode_profile.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32)]
    L.dtgpu_decode_add.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), sz, c,
                                   ctypes.POINTER(ctypes.c_float), ctypes.POINTER(vp)]
    L.dtgpu_decode_add_result.argtypes = [vp, sz, pu64, sz, ctypes.POINTER(sz)]
    L.dtgpu_batch_create_decoded.argtypes = [vp, ctypes.POINTER(vp)]
    L.dtgpu_graph_queries.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(sz), sz,
                                      ctypes.POINTER(GraphQuery), sz, ctypes.POINTER(ctypes.c_int64), sz,
                                      ctypes.POINTER(ctypes.c_int64), sz,
                                      ctypes.POINTER(GraphAnswer), ctypes.POINTER(ctypes.c_float)]
    L.dtgpu_status_str.argtypes = [c]
    L.dtgpu_status_str.restype = ctypes.c_char_p
    _lib = L
    return L


def _check(code):
    if code:
        raise ParseError(code)


def _u64s(xs):
    return (ctypes.c_uint64 * max(1, len(xs)))(*xs), len(xs)


def text_hash(data: bytes) -> int:
    return lib().dtgpu_text_hash(data, len(data))


class ListBranch:
    """Result of a checkout: `ListBranch` (src/list/mod.rs:65-76) content + version."""

    def __init__(self, content: bytes = b"", version=()):
        self._content = content
        self.version = list(version)

    @classmethod
    def new(cls) -> "ListBranch":
        """ListBranch::new() (src/list/branch.rs:12-20): empty content at ROOT."""
        return cls()

    @classmethod
    def new_at_local_version(cls, oplog: "ListOpLog", version) -> "ListBranch":
        """ListBranch::new_at_local_version (src/list/branch.rs:22-26) = oplog.checkout(version)."""
        return oplog.checkout(version)

    @classmethod
    def new_at_tip(cls, oplog: "ListOpLog") -> "ListBranch":
        """ListBranch::new_at_tip (src/list/branch.rs:30-32)."""
        return oplog.checkout_tip()

    def merge(self, oplog: "ListOpLog", merge_frontier) -> None:
        """ListBranch::merge(&mut self, oplog, merge_frontier) (src/list/merge.rs:63-95): apply
        the transformed operations iter_xf_operations_from(self.version, merge_frontier)
        (computed on the GPU) to this branch's content, then move to
        find_dominators_2(self.version, merge_frontier)."""
        v = oplog.dominators(self.version, merge_frontier)
        if v == self.version:
            return
        text = list(self.content())
        for _rng, op in oplog.iter_xf_operations(self.version, merge_frontier):
            if op is None:
                continue
            if op[0] == "ins":
                text[op[1]:op[1]] = list(op[2])
            else:
                del text[op[1]:op[1] + op[2]]
        self._content = "".join(text).encode()
        self.version = v

    def content(self) -> str:
        return self._content.decode("utf-8")

    def content_bytes(self) -> bytes:
        return self._content

    def __len__(self):
        return len(self.content())

    def len(self):
        return len(self)

    def local_frontier(self):
        return list(self.version)


class EncodeOptions(collections.namedtuple(
        "EncodeOptions", "store_inserted_content compress_content store_start_branch_content")):
    """EncodeOptions (src/list/encoding/encode_oplog.rs:88-110): the fields libdtgpu honours
    (user_data, store_deleted_content and the experimental end branch are not offered)."""
    def flags(self):
        return ((1 if self.store_inserted_content else 0) | (2 if self.compress_content else 0)
                | (4 if self.store_start_branch_content else 0))


ENCODE_FULL = EncodeOptions(True, True, True)     # encode_oplog.rs:122-130
ENCODE_PATCH = EncodeOptions(True, True, False)   # encode_oplog.rs:112-120


def lz4_compress(data: bytes) -> bytes:
    """lz4_flex::compress_into as the encoder calls it (encode_oplog.rs:320-343): one raw LZ4
    block, no length prefix."""
    n = ctypes.c_size_t()
    _check(lib().dtgpu_lz4_compress(data, len(data), None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(max(1, n.value))
    _check(lib().dtgpu_lz4_compress(data, len(data), buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


class ListOpLog:
    """Mirror of `ListOpLog` (src/list/mod.rs:103-126) for the checkout path."""

    def __init__(self, _handle=None):
        self._h = _handle if _handle is not None else lib().dtgpu_oplog_new()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().dtgpu_oplog_free(h)
            self._h = None

    @classmethod
    def load_from(cls, data: bytes, ignore_crc: bool = False) -> "ListOpLog":
        out = ctypes.c_void_p()
        _check(lib().dtgpu_oplog_load(data, len(data), int(ignore_crc), ctypes.byref(out)))
        return cls(out.value)

    def decode_and_add(self, data: bytes, ignore_crc: bool = False):
        """ListOpLog::decode_and_add(_opts) (src/list/encoding/decode_oplog.rs:465-583): merge a
        `.dt` file or patch, skipping operations already here; returns the file's version.  On a
        ParseError the oplog is left as it was."""
        cap = 64
        buf = (ctypes.c_uint64 * cap)()
        n = ctypes.c_size_t()
        _check(lib().dtgpu_oplog_decode_and_add(self._h, data, len(data), int(ignore_crc), buf, cap, ctypes.byref(n)))
        if n.value <= cap:
            return list(buf[:n.value])
        # a wider version than the buffer: read the reported frontier back (adds nothing)
        full = (ctypes.c_uint64 * n.value)()
        lib().dtgpu_oplog_last_added_frontier(self._h, full, n.value)
        return list(full)

    @property
    def doc_id(self):
        """ListOpLog::doc_id (src/list/mod.rs:109): None or the document id string."""
        n = lib().dtgpu_oplog_doc_id(self._h, None, 0)
        if n < 0:
            return None
        buf = ctypes.create_string_buffer(max(1, n))
        lib().dtgpu_oplog_doc_id(self._h, buf, n)
        return buf.raw[:n].decode()

    @doc_id.setter
    def doc_id(self, value):
        if value is None:
            _check(lib().dtgpu_oplog_set_doc_id(self._h, None, 0))
        else:
            b = value.encode()
            _check(lib().dtgpu_oplog_set_doc_id(self._h, b, len(b)))

    def __len__(self):
        return lib().dtgpu_oplog_len(self._h)

    def get_or_create_agent_id(self, name: str) -> int:
        b = name.encode()
        a = lib().dtgpu_oplog_get_or_create_agent_id(self._h, b, len(b))
        if a < 0:
            raise ValueError(f"invalid agent name {name!r}")
        return a

    def add_insert_at(self, agent: int, parents, pos: int, content: str) -> int:
        p, n = _u64s(parents)
        b = content.encode()
        return lib().dtgpu_oplog_add_insert_at(self._h, agent, p, n, pos, b, len(b))

    def add_delete_at(self, agent: int, parents, start: int, end: int) -> int:
        p, n = _u64s(parents)
        return lib().dtgpu_oplog_add_delete_at(self._h, agent, p, n, start, end)

    def add_insert(self, agent: int, pos: int, content: str) -> int:
        b = content.encode()
        return lib().dtgpu_oplog_add_insert(self._h, agent, pos, b, len(b))

    def add_delete_without_content(self, agent: int, start: int, end: int) -> int:
        return lib().dtgpu_oplog_add_delete_without_content(self._h, agent, start, end)

    def local_frontier(self):
        buf = (ctypes.c_uint64 * 64)()
        n = lib().dtgpu_oplog_local_frontier(self._h, buf, 64)
        if n > 64:
            buf = (ctypes.c_uint64 * n)()
            lib().dtgpu_oplog_local_frontier(self._h, buf, n)
        return list(buf[:n])

    def plan_stats(self):
        out = (ctypes.c_uint64 * 4)()
        _check(lib().dtgpu_oplog_plan_stats(self._h, out))
        return dict(steps=out[0], retreat=out[1], advance=out[2], commands=out[3])

    def plan_commands(self):
        n = lib().dtgpu_oplog_plan_commands(self._h, None, 0)
        buf = (ctypes.c_uint32 * max(4, 4 * n))()
        lib().dtgpu_oplog_plan_commands(self._h, buf, n)
        return [tuple(buf[4 * i:4 * i + 4]) for i in range(n)]

    def plan_tlist(self):
        n = lib().dtgpu_oplog_plan_tlist(self._h, None, 0)
        buf = (ctypes.c_uint32 * max(1, n))()
        lib().dtgpu_oplog_plan_tlist(self._h, buf, n)
        return list(buf[:n])

    def ins_content(self) -> bytes:
        n = lib().dtgpu_oplog_ins_content(self._h, None, 0)
        buf = ctypes.create_string_buffer(max(1, n))
        lib().dtgpu_oplog_ins_content(self._h, buf, n)
        return buf.raw[:n]

    def char_offsets(self):
        n = lib().dtgpu_oplog_char_offsets(self._h, None, 0)
        buf = (ctypes.c_uint32 * max(1, n))()
        lib().dtgpu_oplog_char_offsets(self._h, buf, n)
        return list(buf[:n])

    def agent_runs(self):
        n = lib().dtgpu_oplog_agent_runs(self._h, None, 0)
        buf = (ctypes.c_uint32 * max(1, n))()
        lib().dtgpu_oplog_agent_runs(self._h, buf, n)
        return list(buf[:n])

    def export(self, what):
        """The decoded oplog's arrays (dtgpu_oplog_export): "ops", "agent_runs", "entries",
        "parent_offsets", "parents", "content", "char_offsets", "version", "agent_names"."""
        a = _export(lambda c, p, n: lib().dtgpu_oplog_export(self._h, c, p, n), what)
        return _names(a) if what == "agent_names" else a

    def cut_ranges(self):
        """Maximal [first, last] LV ranges of cut points (dtgpu_oplog_cut_ranges): v such that the
        ops below v are the version {v-1} and every later op has v-1 in its history."""
        n = lib().dtgpu_oplog_cut_ranges(self._h, None, 0)
        buf = (ctypes.c_uint64 * max(2, 2 * n))()
        lib().dtgpu_oplog_cut_ranges(self._h, buf, n)
        return [(int(buf[2 * k]), int(buf[2 * k + 1])) for k in range(n)]

    def checkout_tip_bytes(self) -> bytes:
        n = ctypes.c_size_t()
        _check(lib().dtgpu_checkout_tip(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(lib().dtgpu_checkout_tip(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def checkout_tip(self) -> ListBranch:
        return ListBranch(self.checkout_tip_bytes(), self.local_frontier())

    def xf_order(self, frm=None, merging=None):
        """LV order of iter_xf_operations(_from) (host plan: fast-forward prefix, then the
        walker); default ROOT to the tip."""
        if frm is None and merging is None:
            frm, merging = [], self.local_frontier()
        pa, na = _u64s(frm or [])
        pb, nb = _u64s(merging or [])
        n = len(self)
        buf = (ctypes.c_uint32 * max(1, n))()
        k = lib().dtgpu_oplog_xf_order(self._h, pa, na, pb, nb, buf, n)
        return list(buf[:k])

    def xf_operations_lv(self, frm=None, merging=None):
        """Per-LV transformed positions in application order, computed on the GPU
        (dtgpu_xf_operations_from; default: ROOT to the tip): [(lv, pos or None)], None =
        DeleteAlreadyHappened."""
        if frm is None and merging is None:
            frm, merging = [], self.local_frontier()
        pa, na = _u64s(frm or [])
        pb, nb = _u64s(merging or [])
        k = ctypes.c_size_t()
        _check(lib().dtgpu_xf_operations_from(self._h, pa, na, pb, nb, None, 0, ctypes.byref(k)))
        n = k.value
        buf = (ctypes.c_uint32 * max(2, 2 * n))()
        _check(lib().dtgpu_xf_operations_from(self._h, pa, na, pb, nb, buf, n, ctypes.byref(k)))
        return [(buf[2 * i], None if buf[2 * i + 1] == 0xFFFFFFFF else buf[2 * i + 1]) for i in range(k.value)]

    def iter_xf_operations_from(self, frm, merging):
        """ListOpLog::iter_xf_operations_from (src/list/merge.rs:24-38); see iter_xf_operations."""
        return self.iter_xf_operations(frm, merging)

    def iter_xf_operations(self, frm=None, merging=None):
        """ListOpLog::iter_xf_operations() (src/list/merge.rs:40-48): yields (range(lv, lv+len),
        op) with op = ("ins", pos, text) / ("del", pos, len) / None (DeleteAlreadyHappened).
        Consecutive LVs of one op run are merged when they form one reference-style op: an
        insert at consecutive positions, a forward delete at one position, a backspace run at
        descending positions (reported at its lowest position, like BaseMoved)."""
        ops = self.export("ops").reshape(-1, 4)
        content = self.ins_content()
        coff = self.char_offsets()
        run_of = {}
        for r, (lv, ln, _pos, kf) in enumerate(ops):
            for k in range(int(ln)):
                run_of[int(lv) + k] = (r, int(kf) & 1)

        def char(v):
            b = coff[v]
            n = 1 if content[b] < 0x80 else 2 if content[b] < 0xE0 else 3 if content[b] < 0xF0 else 4
            return content[b:b + n].decode("utf-8")

        cur = None   # [start_lv, end_lv, run, kind, first_pos, last_pos, text, step]
        for lv, x in self.xf_operations_lv(frm, merging):
            r, kind = run_of[lv]
            if cur is not None and lv == cur[1] and r == cur[2]:
                if x is None and cur[3] is None:
                    cur[1] += 1
                    continue
                if x is not None and cur[3] == kind:
                    step = x - cur[5]
                    want = {0: (1,), 1: (0, -1)}[kind] if cur[7] is None else (cur[7],)
                    if step in want and (kind == 0 or cur[1] - cur[0] == 1 or step == cur[7]):
                        cur[1] += 1
                        cur[5] = x
                        cur[7] = step
                        if kind == 0:
                            cur[6] += char(lv)
                        continue
            if cur is not None:
                yield self._xf_item(cur)
            cur = [lv, lv + 1, r, None if x is None else kind, x, x, char(lv) if (x is not None and kind == 0) else "", None]
        if cur is not None:
            yield self._xf_item(cur)

    @staticmethod
    def _xf_item(cur):
        rng = range(cur[0], cur[1])
        if cur[3] is None:
            return rng, None
        if cur[3] == 0:
            return rng, ("ins", cur[4], cur[6])
        return rng, ("del", min(cur[4], cur[5]), cur[1] - cur[0])

    def encode(self, opts=None) -> bytes:
        """ListOpLog::encode(opts) (src/list/encoding/encode_oplog.rs:745-747); opts defaults to
        ENCODE_FULL (EncodeOptions::default, :133-137)."""
        return self.encode_from([], opts)

    def encode_from(self, frm, opts=None) -> bytes:
        """ListOpLog::encode_from(opts, from) (encode_oplog.rs:404-743): the ops after version
        `frm`.  With opts.store_start_branch_content and a non-ROOT `frm`, the StartBranch holds
        the checkout at `frm`, run on the GPU."""
        p, nf = _u64s(frm)
        flags = (opts or ENCODE_FULL).flags()
        n = ctypes.c_size_t()
        _check(lib().dtgpu_oplog_encode(self._h, p, nf, flags, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(lib().dtgpu_oplog_encode(self._h, p, nf, flags, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def dominators(self, a, b=()):
        """Graph::find_dominators_2 (src/causalgraph/graph/tools.rs:545-578) over this oplog."""
        pa, na = _u64s(a)
        pb, nb = _u64s(b)
        cap = na + nb + 1
        out = (ctypes.c_uint64 * cap)()
        n = lib().dtgpu_oplog_dominators(self._h, pa, na, pb, nb, out, cap)
        if n < 0:
            raise ValueError("version names an LV outside the oplog")
        return list(out[:n])

    def checkout_bytes(self, version) -> bytes:
        p, nv = _u64s(version)
        n = ctypes.c_size_t()
        _check(lib().dtgpu_checkout(self._h, p, nv, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(lib().dtgpu_checkout(self._h, p, nv, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def history(self, version) -> "ListOpLog":
        """The history of `version` as its own oplog (dtgpu_oplog_history)."""
        p, nv = _u64s(version)
        out = ctypes.c_void_p()
        _check(lib().dtgpu_oplog_history(self._h, p, nv, ctypes.byref(out)))
        return ListOpLog(out.value)

    def project(self, spans) -> "ListOpLog":
        """The ops in the LV spans [(start, end), ...] with the causal graph projected onto them
        (Graph::subgraph_raw, src/causalgraph/graph/subgraph.rs:39-250; dtgpu_oplog_project)."""
        flat = [int(x) for s in spans for x in s]
        p = (ctypes.c_uint64 * max(1, len(flat)))(*flat)
        out = ctypes.c_void_p()
        _check(lib().dtgpu_oplog_project(self._h, p, len(flat) // 2, ctypes.byref(out)))
        return ListOpLog(out.value)

    def project_version(self, spans, version):
        """A version of this oplog projected onto the sub-oplog of `spans` (the numbering
        `project(spans)` gives): the frontier of Hist(version) n spans
        (Graph::project_onto_subgraph_raw; dtgpu_oplog_project_version)."""
        flat = [int(x) for s in spans for x in s]
        p = (ctypes.c_uint64 * max(1, len(flat)))(*flat)
        pv, nv = _u64s(version)
        cap = max(1, len(flat))
        out = (ctypes.c_uint64 * cap)()
        n = lib().dtgpu_oplog_project_version(self._h, p, len(flat) // 2, pv, nv, out, cap)
        if n < 0:
            raise ValueError("bad spans or version")
        if n > cap:
            out = (ctypes.c_uint64 * n)()
            n = lib().dtgpu_oplog_project_version(self._h, p, len(flat) // 2, pv, nv, out, n)
        return list(out[:n])

    def local_to_remote(self, lv):
        """AgentAssignment::local_to_agent_version: LV -> (agent id, seq)."""
        a, q = ctypes.c_uint32(), ctypes.c_uint64()
        _check(lib().dtgpu_oplog_local_to_remote(self._h, lv, ctypes.byref(a), ctypes.byref(q)))
        return a.value, q.value

    def remote_to_local(self, agent, seq, n=1):
        """Local LV spans [(start, end)] of the remote span (agent id, seq .. seq + n), in seq
        order; KeyError when part of it is unknown here."""
        cap = 8
        while True:
            buf = (ctypes.c_uint64 * (2 * cap))()
            k = lib().dtgpu_oplog_remote_to_local(self._h, agent, seq, n, buf, cap)
            if k < 0:
                raise KeyError((agent, seq, n))
            if k <= cap:
                return [(buf[2 * i], buf[2 * i + 1]) for i in range(k)]
            cap = k

    def checkout_text_bytes(self, spans) -> bytes:
        """OpLog::checkout_text (src/oplog.rs:388-394) for the text whose ops are `spans`: the
        projected sub-oplog checked out on the device."""
        return self.project(spans).checkout_tip_bytes()

    def checkout(self, version) -> ListBranch:
        """ListOpLog::checkout(&[LV]) (src/list/oplog.rs:32-36): the branch at `version`."""
        v = self.dominators(version)
        return ListBranch(self.checkout_bytes(v), v)


# dtgpu_export codes (include/dtgpu.h): name -> (code, numpy dtype, fields per record)
EXPORTS = {
    "ops": (0, "<u4", 4), "agent_runs": (1, "<u4", 4), "entries": (2, "<u4", 2),
    "parent_offsets": (3, "<u4", 1), "parents": (4, "<u4", 1), "content": (5, "u1", 1),
    "char_offsets": (6, "<u4", 1), "version": (7, "<u4", 1), "agent_names": (8, "u1", 1),
    "doc_id": (9, "u1", 1),
}
DECODE_DEFER = 80


def _export(fn, what):
    import numpy as np
    code, dt, per = EXPORTS[what]
    n = fn(code, None, 0)
    arr = np.zeros(max(n, 1) * per, dtype=dt)
    fn(code, arr.ctypes.data_as(ctypes.c_void_p), n)
    arr = arr[:n * per]
    return arr.reshape(n, per) if per > 1 else arr


def _names(blob):
    out, i = [], 0
    blob = bytes(blob)
    while i < len(blob):
        k = blob[i]
        out.append(blob[i + 1:i + 1 + k])
        i += 1 + k
    return out


def oplog_from_trace(txns, agent_name="jeremy") -> ListOpLog:
    """crates/bench/src/utils.rs:25-44 apply_edits_push_merge (delete then insert per patch)."""
    o = ListOpLog()
    a = o.get_or_create_agent_id(agent_name)
    for txn in txns:
        for pos, dl, ins in txn["patches"]:
            if dl > 0:
                o.add_delete_without_content(a, pos, pos + dl)
            if ins:
                o.add_insert(a, pos, ins)
    return o


class Batch:
    """A batch staged in HBM.  staging="host": decode and planner inputs on host threads;
    staging="device": `.dt` bytes to HBM, then decode (dt_decode.hip) and planner inputs
    (dt_prep.hip) on the GPU as well.  Walk planning (dt_plan.hip), replay and materialisation
    (dt_replay.hip) always run on the GPU."""

    def __init__(self, docs=None, oplogs=None, ignore_crc=False, host_threads=0, device=0, staging="host",
                 xf=False, flags=0, seg_ops=0, seg_max=0, lds_fill=0):
        """xf=True (with oplogs): a transformed-ops batch, every document's iter_xf_operations()
        computed by the replay (dtgpu_batch_create_xf); read it with xf_positions(i).  flags
        (OPT_*), seg_ops, seg_max, lds_fill: dtgpu_batch_opts."""
        L = lib()
        opts = BatchOpts(int(ignore_crc), int(host_threads), int(device), int(flags), int(seg_ops), int(seg_max),
                         int(lds_fill))
        out = ctypes.c_void_p()
        if oplogs is not None:
            arr = (ctypes.c_void_p * max(1, len(oplogs)))(*[o._h for o in oplogs])
            self._keep = oplogs
            create = L.dtgpu_batch_create_xf if xf else L.dtgpu_batch_create_from_oplogs
            _check(create(arr, len(oplogs), ctypes.byref(opts), ctypes.byref(out)))
            self.n = len(oplogs)
        else:
            self._keep = list(docs)
            ptrs = (ctypes.c_char_p * max(1, len(self._keep)))(*self._keep)
            lens = (ctypes.c_size_t * max(1, len(self._keep)))(*[len(d) for d in self._keep])
            create = L.dtgpu_batch_create_device if staging == "device" else L.dtgpu_batch_create
            _check(create(ptrs, lens, len(self._keep), ctypes.byref(opts), ctypes.byref(out)))
            self.n = len(self._keep)
        self._h = out.value

    def __len__(self):
        return self.n

    def xf_positions(self, i):
        """Per-LV BaseMoved positions of document i (xf batches; None = DeleteAlreadyHappened)."""
        k = ctypes.c_size_t()
        _check(lib().dtgpu_batch_xf_positions(self._h, i, None, 0, ctypes.byref(k)))
        buf = (ctypes.c_uint32 * max(1, k.value))()
        _check(lib().dtgpu_batch_xf_positions(self._h, i, buf, k.value, ctypes.byref(k)))
        return [None if x == 0xFFFFFFFF else x for x in buf[:k.value]]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().dtgpu_batch_free(h)
            self._h = None

    def run(self, stream=None):
        _check(lib().dtgpu_batch_run(self._h, stream))

    def run_timed(self) -> float:
        ms = ctypes.c_float()
        _check(lib().dtgpu_batch_run_timed(self._h, ctypes.byref(ms)))
        return ms.value

    def run_e2e_timed(self):
        """Device-staged batches: decode + prep + plan + replay again; kernel ms of each."""
        ms = (ctypes.c_float * 4)()
        _check(lib().dtgpu_batch_run_e2e_timed(self._h, ms))
        return list(ms)

    def encode(self, opts=None) -> float:
        """Device-staged batches: ListOpLog::encode(opts) from ROOT for every document on the GPU
        (dtgpu_batch_encode); returns the encode kernel's ms.  Read the bytes with encoded(i)."""
        ms = ctypes.c_float()
        _check(lib().dtgpu_batch_encode(self._h, (opts or ENCODE_FULL).flags(), ctypes.byref(ms)))
        return ms.value

    def encoded(self, i) -> bytes:
        n = ctypes.c_size_t()
        _check(lib().dtgpu_batch_encoded(self._h, i, None, 0, ctypes.byref(n), None))
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(lib().dtgpu_batch_encoded(self._h, i, buf, n.value, ctypes.byref(n), None))
        return buf.raw[:n.value]

    def encoded_status(self, i) -> int:
        n = ctypes.c_size_t()
        return lib().dtgpu_batch_encoded(self._h, i, None, 0, ctypes.byref(n), None)

    def encode_profile(self, i):
        n = ctypes.c_size_t()
        out = (ctypes.c_uint64 * 14)()
        _check(lib().dtgpu_batch_encoded(self._h, i, None, 0, ctypes.byref(n), out))
        return dict(zip(["walk", "op_runs", "sizes", "text_lz4", "write", "crc", "lz_probe", "lz_extend",
                         "lz_emit", "lz_steps", "lz_shared_steps", "lz_sequences", "txn_heads", "agent_runs"], list(out)))

    def encoded_bytes(self, which=0) -> int:
        return lib().dtgpu_batch_encoded_bytes(self._h, which)

    def sync(self):
        _check(lib().dtgpu_batch_sync(self._h))

    def results(self):
        arr = (DocResult * max(1, self.n))()
        _check(lib().dtgpu_batch_results(self._h, arr))
        return [dict(status=r.status, text_len=r.text_len, text_hash=r.text_hash, n_lv=r.n_lv) for r in arr[:self.n]]

    def text(self, i) -> bytes:
        n = ctypes.c_size_t()
        _check(lib().dtgpu_batch_text(self._h, i, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(lib().dtgpu_batch_text(self._h, i, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def last_times(self):
        """(plan_ms, replay_ms, prep_ms) of the last run_timed() (prep_ms 0 when host-staged)."""
        out = (ctypes.c_float * 3)()
        _check(lib().dtgpu_batch_last_times(self._h, out))
        return out[0], out[1], out[2]

    def host_planned(self):
        n = len(self)
        buf = (ctypes.c_uint8 * max(1, n))()
        lib().dtgpu_batch_host_planned(self._h, buf, n)
        return [int(x) for x in buf[:n]]

    def fast_forwarded(self):
        """Per document: 1 when it checked out on the fast-forward path (dt_ff.hip: a linear
        history, merge.rs:811-840), else 0."""
        n = len(self)
        buf = (ctypes.c_uint8 * max(1, n))()
        lib().dtgpu_batch_fast_forwarded(self._h, buf, n)
        return [int(x) for x in buf[:n]]

    def plan(self, i):
        """Command stream (op, lv, len, pos) and retreat/advance entries of document i."""
        nc, nt = ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib().dtgpu_batch_plan(self._h, i, None, 0, None, 0, ctypes.byref(nc), ctypes.byref(nt)))
        cb = (ctypes.c_uint32 * max(4, 4 * nc.value))()
        tb = (ctypes.c_uint32 * max(1, nt.value))()
        _check(lib().dtgpu_batch_plan(self._h, i, cb, nc.value, tb, nt.value, ctypes.byref(nc), ctypes.byref(nt)))
        return [tuple(cb[4 * k:4 * k + 4]) for k in range(nc.value)], list(tb[:nt.value])

    def plan_profile(self, i):
        out = (ctypes.c_uint64 * 8)()
        _check(lib().dtgpu_batch_plan_profile(self._h, i, out))
        keys = ["rec", "parents", "children", "emit", "ops", "init", "n_cmds", "n_tlist"]
        return dict(zip(keys, list(out)))

    def doc_stats(self, i):
        """Diagnostics of document i after a run (see dtgpu_batch_doc_stats)."""
        out = (ctypes.c_uint32 * 29)()
        _check(lib().dtgpu_batch_doc_stats(self._h, i, out))
        keys = ["n_items", "n_blocks", "fail_cmd", "fail_site", "n_cmds", "max_blocks",
                "cyc_ins", "cyc_del", "cyc_tog", "cyc_mat", "cyc_yjs", "cyc_split", "cyc_find", "cyc_bload",
                "cyc_orr", "cyc_run", "cyc_r1", "cyc_r2", "cyc_r3", "n_yjs", "n_split", "cyc_total",
                "n_sb", "lds_index", "cyc_t1", "cyc_t2", "cyc_t3", "n_dirty", "n_load"]
        return dict(zip(keys, list(out)))

    def segments(self, i):
        """Cut replay: the LV segments document i replayed as (see dtgpu_batch_segments), as
        dicts; [] when it replayed whole."""
        out = (ctypes.c_uint32 * (12 * 64))()
        n = lib().dtgpu_batch_segments(self._h, i, out, 64)
        keys = ["lo", "hi", "placeholders", "status", "items_visible", "cyc_total", "lds_index", "n_blocks",
                "host_fallback", "host_lo", "host_hi", "host_placeholders"]
        return [dict(zip(keys, list(out[12 * k:12 * k + 12]))) for k in range(min(n, 64))]

    @property
    def algorithmic_bytes(self):
        return lib().dtgpu_batch_algorithmic_bytes(self._h)

    @property
    def total_lv(self):
        return lib().dtgpu_batch_total_lv(self._h)


class DecodeBatch:
    """Batched `ListOpLog::load_from` on the GPU (dtgpu_decode_*): one wavefront per document."""

    def __init__(self, docs, ignore_crc=False, device=0):
        L = lib()
        n = len(docs)
        self._keep = [bytes(d) for d in docs]
        arr = (ctypes.c_char_p * max(n, 1))(*self._keep)
        lens = (ctypes.c_size_t * max(n, 1))(*[len(d) for d in self._keep])
        opts = BatchOpts(1 if ignore_crc else 0, 0, device)
        h = ctypes.c_void_p()
        _check(L.dtgpu_decode_create(arr, lens, n, ctypes.byref(opts), ctypes.byref(h)))
        self._h = h
        self.n = n

    def __len__(self):
        return self.n

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().dtgpu_decode_free(h)
            self._h = None

    def run(self) -> float:
        """Full device decode of every document; returns the kernel time in ms."""
        ms = ctypes.c_float()
        _check(lib().dtgpu_decode_run(self._h, ctypes.byref(ms)))
        return ms.value

    def status(self, i):
        out = (ctypes.c_uint64 * 12)()
        _check(lib().dtgpu_decode_status(self._h, i, out))
        keys = ("status", "n_lv", "n_ops", "n_aruns", "n_entries", "n_parents", "n_content", "n_version",
                "n_agents", "content_complete", "ascii", "n_file_agents")
        return dict(zip(keys, list(out)))

    def export(self, i, what):
        a = _export(lambda c, p, n: lib().dtgpu_decode_export(self._h, i, c, p, n), what)
        return _names(a) if what == "agent_names" else a

    def doc_id(self, i):
        a = bytes(self.export(i, "doc_id"))
        return a[1:].decode() if a and a[0] else None

    def add(self, patches, ignore_crc=False):
        """ListOpLog::decode_and_add of patches[i] into document i, on the GPU (dtgpu_decode_add):
        a new DecodeBatch of the merged oplogs (this one is unchanged).  Per-document outcome:
        add_result(i)."""
        n = len(patches)
        keep = [bytes(p) for p in patches]
        arr = (ctypes.c_char_p * max(n, 1))(*keep)
        lens = (ctypes.c_size_t * max(n, 1))(*[len(p) for p in keep])
        ms = ctypes.c_float()
        h = ctypes.c_void_p()
        _check(lib().dtgpu_decode_add(self._h, arr, lens, n, int(ignore_crc), ctypes.byref(ms), ctypes.byref(h)))
        m = DecodeBatch.__new__(DecodeBatch)
        m._h, m.n, m._keep, m.last_ms = h, n, keep, ms.value
        return m

    def add_result(self, i):
        """(status, the patch's version): decode_and_add's Result for document i of a merged batch."""
        k = ctypes.c_size_t()
        buf = (ctypes.c_uint64 * 64)()
        st = lib().dtgpu_decode_add_result(self._h, i, buf, 64, ctypes.byref(k))
        return st, list(buf[:k.value])

    def checkout_batch(self):
        """A device-staged checkout Batch over these decoded (or merged) oplogs; consumes this
        handle (dtgpu_batch_create_decoded)."""
        h, self._h = self._h, None
        b = Batch.__new__(Batch)
        out = ctypes.c_void_p()
        _check(lib().dtgpu_batch_create_decoded(h, ctypes.byref(out)))
        b._h, b.n, b._keep = out.value, self.n, None
        return b

    def profile(self, i):
        out = (ctypes.c_uint32 * 8)()
        _check(lib().dtgpu_decode_profile(self._h, i, out))
        return list(out)

    def bytes_in(self) -> int:
        return lib().dtgpu_decode_bytes(self._h, 0)

    def bytes_out(self) -> int:
        return lib().dtgpu_decode_bytes(self._h, 1)


GQ_KINDS = {"diff": 0, "conflict": 1, "contains": 2, "dominators": 3, "diff_level": 4, "conflict_level": 5}
DIFF_FLAGS = ["OnlyA", "OnlyB", "Shared"]


def graph_queries(graphs, queries, span_cap=512, timing=False, common_cap=None):
    """Batched causal-graph queries on the GPU (dtgpu_graph_queries, one wavefront per query).

    graphs: GraphEntrySimple lists ([{"span": [start, end], "parents": [...]}, ...]).
    queries: ("diff", g, a, b) -> (only_a, only_b) span lists, newest first (Graph::diff_rev);
             ("conflict", g, a, b) -> ([(start, end, flag)], common) (Graph::find_conflicting);
             ("contains", g, frontier, target) -> bool (frontier_contains_version; -1 = ROOT);
             ("dominators", g, a, b) -> sorted list (find_dominators_2 of two dominator sets);
             ("diff_level", g, a, b) -> as "diff", by level-synchronous propagation (dt_level.hip);
             ("conflict_level", g, a, b) -> as "conflict": level-synchronous marks + a bucketed sweep.
    Frontiers may be of any width.  A query the device could not answer yields ("error", status)."""
    hist, off = [], [0]
    for g in graphs:
        for e in g:
            hist += [e["span"][0], e["span"][1], len(e["parents"])] + list(e["parents"])
        off.append(len(hist))
    H = (ctypes.c_int64 * max(1, len(hist)))(*hist)
    O = (ctypes.c_size_t * len(off))(*off)
    nq = len(queries)
    Q = (GraphQuery * max(1, nq))()
    keep = []   # the frontier arrays the query structs point at
    for i, (kind, g, a, b) in enumerate(queries):
        q = Q[i]
        q.kind, q.graph, q.na = GQ_KINDS[kind], g, len(a)
        fa = (ctypes.c_int64 * max(1, len(a)))(*a)
        keep.append(fa)
        q.a = ctypes.cast(fa, ctypes.POINTER(ctypes.c_int64))
        if kind == "contains":
            q.target = b
        else:
            q.nb = len(b)
            fb = (ctypes.c_int64 * max(1, len(b)))(*b)
            keep.append(fb)
            q.b = ctypes.cast(fb, ctypes.POINTER(ctypes.c_int64))
    if common_cap is None:   # room for any answer: a common frontier / dominator set is never
        common_cap = max([2] + [len(a) + (0 if k == "contains" else len(b)) + 1 for k, _g, a, b in queries]
                         + [max([len(e["parents"]) for e in gr] or [0]) + 1 for gr in graphs])
    spans = (ctypes.c_int64 * (max(1, nq) * span_cap * 3))()
    common = (ctypes.c_int64 * (max(1, nq) * common_cap))()
    ans = (GraphAnswer * max(1, nq))()
    ms = ctypes.c_float()
    _check(lib().dtgpu_graph_queries(H, O, len(graphs), Q, nq, spans, span_cap, common, common_cap, ans,
                                     ctypes.byref(ms)))
    out = []
    for i, (kind, _g, _a, _b) in enumerate(queries):
        r = ans[i]
        if r.status:
            out.append(("error", r.status))
            continue
        base = 3 * span_cap * i
        tri = [(spans[base + 3 * k], spans[base + 3 * k + 1], spans[base + 3 * k + 2]) for k in range(r.n_a + r.n_b)]
        if kind in ("diff", "diff_level"):
            out.append(([(s, e) for s, e, _ in tri[:r.n_a]], [(s, e) for s, e, _ in tri[r.n_a:]]))
        elif kind in ("conflict", "conflict_level"):
            cb = common_cap * i
            out.append(([(s, e, DIFF_FLAGS[f]) for s, e, f in tri[:r.n_a]], list(common[cb:cb + r.n_common])))
        elif kind == "dominators":
            cb = common_cap * i
            out.append(list(common[cb:cb + r.n_common]))
        else:
            out.append(bool(r.n_a))
    return (out, ms.value) if timing else out


def batch_checkout(docs, **kw):
    """Checkout every `.dt` document in `docs`; returns (results, texts)."""
    b = Batch(docs=docs, **kw)
    b.run()
    b.sync()
    res = b.results()
    return res, [b.text(i) if r["status"] == 0 else None for i, r in enumerate(res)]


def device_count() -> int:
    return lib().dtgpu_device_count()


def synth_ops(doc, target_ops=5000):
    """Op list of synthetic document `doc` (dt_synth.cpp): (n_agents, [(agent, kind, pos, len,
    text, parents)])."""
    na = ctypes.c_uint32()
    n = lib().dtgpu_synth_ops(doc, target_ops, ctypes.byref(na), None, 0)
    buf = (ctypes.c_uint32 * max(1, n))()
    lib().dtgpu_synth_ops(doc, target_ops, ctypes.byref(na), buf, n)
    w = list(buf[:n])
    ops, i = [], 0
    while i < n:
        agent, kind, pos, ln, c0, c1, np_ = w[i:i + 7]
        text = bytes([c0, c1][:ln]).decode() if kind == 0 else ""
        ops.append((agent, kind, pos, ln, text, w[i + 7:i + 7 + np_]))
        i += 7 + np_
    return na.value, ops


def synth_oplog(doc, target_ops=5000):
    """Synthetic document `doc` built as a ListOpLog."""
    h = ctypes.c_void_p()
    _check(lib().dtgpu_synth_oplog(doc, target_ops, ctypes.byref(h)))
    return ListOpLog(h.value)


def synth_merge_oplog(doc, target_ops=5000, n_agents=0):
    """SURVEY.md 8(d)4 synthetic document `doc` (dt_synth.cpp MergeGen: per-step pairwise merges
    with p = 0.1 via find_dominators_2, make_random_change edits), built as a ListOpLog.
    n_agents = 0 draws U{4..16}; a larger count gives a wide history (many causal chains)."""
    h = ctypes.c_void_p()
    _check(lib().dtgpu_synth_merge_oplog(doc, target_ops, n_agents, ctypes.byref(h)))
    return ListOpLog(h.value)


def apply_edits_push_merge(txns, agent_name="jeremy"):
    """crates/bench/src/utils.rs:25-44 (apply_edits_push_merge): a JSON trace's patches
    (pos, del, ins) pushed into a new ListOpLog by one agent at the current version, delete
    before insert.  The oplog the reference's benches and checkout_tip run on."""
    o = ListOpLog()
    a = o.get_or_create_agent_id(agent_name)
    for txn in txns:
        for pos, dl, ins in txn["patches"]:
            if dl:
                o.add_delete_without_content(a, pos, pos + dl)
            if ins:
                o.add_insert(a, pos, ins)
    return o
