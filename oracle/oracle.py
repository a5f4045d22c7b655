"""ctypes binding of the CPU oracle (oracle/dt_oracle.c).

TEST INFRASTRUCTURE ONLY.  This module is the parity checker for the MI355X engine: only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.  The product
(diamond-types_amd/dt_amd, libdtgpu.so) never imports or links it.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

i64 = ctypes.c_int64
P64 = ctypes.POINTER(ctypes.c_int64)


class Stats(ctypes.Structure):
    _fields_ = [("n_steps", i64), ("n_retreat", i64), ("n_advance", i64), ("n_scans", i64), ("n_items", i64)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.dto_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.dto_new.restype = ctypes.c_void_p
        L.dto_free.argtypes = [ctypes.c_void_p]
        L.dto_len.argtypes = [ctypes.c_void_p]
        L.dto_len.restype = i64
        L.dto_get_or_create_agent.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.dto_add_insert_at.argtypes = [ctypes.c_void_p, ctypes.c_int, P64, ctypes.c_int, i64, ctypes.c_char_p, i64]
        L.dto_add_insert_at.restype = i64
        L.dto_add_delete_at.argtypes = [ctypes.c_void_p, ctypes.c_int, P64, ctypes.c_int, i64, i64]
        L.dto_add_delete_at.restype = i64
        L.dto_add_insert.argtypes = [ctypes.c_void_p, ctypes.c_int, i64, ctypes.c_char_p, i64]
        L.dto_add_insert.restype = i64
        L.dto_add_delete.argtypes = [ctypes.c_void_p, ctypes.c_int, i64, i64]
        L.dto_add_delete.restype = i64
        L.dto_frontier.argtypes = [ctypes.c_void_p, P64, ctypes.c_int]
        L.dto_num_agents.argtypes = [ctypes.c_void_p]
        L.dto_num_graph_entries.argtypes = [ctypes.c_void_p]
        L.dto_num_graph_entries.restype = i64
        L.dto_num_agent_runs.argtypes = [ctypes.c_void_p]
        L.dto_num_agent_runs.restype = i64
        L.dto_ins_content_len.argtypes = [ctypes.c_void_p]
        L.dto_ins_content_len.restype = i64
        L.dto_checkout_tip.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(Stats)]
        L.dto_checkout.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(Stats)]
        L.dto_free_buf.argtypes = [ctypes.c_void_p]
        for f in ("dto_export_lv", "dto_export_aruns", "dto_export_version"):
            getattr(L, f).argtypes = [ctypes.c_void_p, P64, i64]
            getattr(L, f).restype = i64
        L.dto_export_entries.argtypes = [ctypes.c_void_p, P64, i64, P64, i64]
        L.dto_export_entries.restype = i64
        L.dto_agent_name.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.dto_agent_name.restype = ctypes.c_int
        L.dto_ins_content.argtypes = [ctypes.c_void_p]
        L.dto_ins_content.restype = ctypes.c_void_p
        L.dto_checkout_tip_ff.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int)]
        L.dto_xf_operations.argtypes = [ctypes.c_void_p, P64]
        L.dto_xf_operations_from.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, P64, ctypes.c_int, P64, P64]
        L.dto_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.dto_crc32c.restype = ctypes.c_uint32
        L.dto_lz4_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.dto_graph_new.restype = ctypes.c_void_p
        L.dto_graph_free.argtypes = [ctypes.c_void_p]
        L.dto_graph_push.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, i64, i64]
        L.dto_graph_num_entries.argtypes = [ctypes.c_void_p]
        L.dto_graph_entry.argtypes = [ctypes.c_void_p, ctypes.c_int, P64, P64, P64]
        L.dto_graph_diff.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, P64, ctypes.c_int,
                                     P64, ctypes.POINTER(ctypes.c_int), P64, ctypes.POINTER(ctypes.c_int)]
        L.dto_graph_contains.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, i64]
        L.dto_graph_dominators.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, P64, ctypes.c_int, P64]
        L.dto_graph_find_conflicting.argtypes = [ctypes.c_void_p, P64, ctypes.c_int, P64, ctypes.c_int,
                                                 P64, P64, ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def _arr(xs):
    a = (ctypes.c_int64 * max(1, len(xs)))(*xs)
    return a, len(xs)


class OracleError(Exception):
    def __init__(self, code):
        super().__init__(f"oracle error {code}")
        self.code = code


class OpLog:
    """Mirror of the reference `ListOpLog` surface the tests need (src/list/oplog.rs)."""

    def __init__(self, handle=None):
        self.h = handle if handle is not None else lib().dto_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().dto_free(self.h)
            self.h = None

    @classmethod
    def load_from(cls, data: bytes, ignore_crc=False):
        out = ctypes.c_void_p()
        e = lib().dto_load(data, len(data), int(ignore_crc), ctypes.byref(out))
        if e:
            raise OracleError(e)
        return cls(out.value)

    def __len__(self):
        return lib().dto_len(self.h)

    def agent(self, name: str) -> int:
        b = name.encode()
        return lib().dto_get_or_create_agent(self.h, b, len(b))

    def add_insert_at(self, agent, parents, pos, content: str):
        a, n = _arr(parents)
        b = content.encode()
        return lib().dto_add_insert_at(self.h, agent, a, n, pos, b, len(b))

    def add_delete_at(self, agent, parents, start, end):
        a, n = _arr(parents)
        return lib().dto_add_delete_at(self.h, agent, a, n, start, end)

    def add_insert(self, agent, pos, content: str):
        b = content.encode()
        return lib().dto_add_insert(self.h, agent, pos, b, len(b))

    def add_delete(self, agent, start, end):
        return lib().dto_add_delete(self.h, agent, start, end)

    def frontier(self):
        buf = (ctypes.c_int64 * 256)()
        n = lib().dto_frontier(self.h, buf, 256)
        return list(buf[:n])

    def checkout_tip_bytes(self, order=0, with_stats=False):
        out = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        st = Stats()
        e = lib().dto_checkout_tip(self.h, order, ctypes.byref(out), ctypes.byref(ln), ctypes.byref(st))
        if e:
            raise OracleError(e)
        data = ctypes.string_at(out.value, ln.value) if ln.value else b""
        lib().dto_free_buf(out)
        if with_stats:
            return data, {k: getattr(st, k) for k, _ in Stats._fields_}
        return data

    def decoded(self):
        """The oracle's decoded arrays (independent restatement of decode_internal): per-LV
        (kind, pos, cbyte) triples, agent runs, graph entries (start, end, parents), version,
        agent names and inserted content."""
        L = lib()

        def grab(fn, per, *extra):
            n = fn(self.h, None, 0, *extra)
            buf = (ctypes.c_int64 * max(1, per * n))()
            fn(self.h, buf, n, *extra)
            return [tuple(buf[per * i:per * i + per]) for i in range(n)]
        lvs = grab(L.dto_export_lv, 3)
        aruns = grab(L.dto_export_aruns, 4)
        ne = L.dto_export_entries(self.h, None, 0, None, 0)
        eb = (ctypes.c_int64 * max(1, 3 * ne))()
        L.dto_export_entries(self.h, eb, ne, None, 0)
        npar = sum(eb[3 * i + 2] for i in range(ne))
        pb = (ctypes.c_int64 * max(1, npar))()
        L.dto_export_entries(self.h, eb, ne, pb, npar)
        entries, k = [], 0
        for i in range(ne):
            np_ = eb[3 * i + 2]
            entries.append((eb[3 * i], eb[3 * i + 1], tuple(pb[k:k + np_])))
            k += np_
        nv = L.dto_export_version(self.h, None, 0)
        vb = (ctypes.c_int64 * max(1, nv))()
        L.dto_export_version(self.h, vb, nv)
        names = []
        for i in range(L.dto_num_agents(self.h)):
            n = L.dto_agent_name(self.h, i, None, 0)
            nb = ctypes.create_string_buffer(max(1, n))
            L.dto_agent_name(self.h, i, nb, n)
            names.append(nb.raw[:n].decode())
        clen = L.dto_ins_content_len(self.h)
        content = ctypes.string_at(L.dto_ins_content(self.h), clen) if clen else b""
        return {"lv": lvs, "agent_runs": aruns, "entries": entries, "version": list(vb[:nv]),
                "agent_names": names, "content": content}

    def checkout_tip_ff_bytes(self):
        """checkout_tip with the reference's fast-forward path for linear histories
        (merge.rs:811-840); (text, ff) with ff True when no tracker was needed."""
        out = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        ff = ctypes.c_int()
        e = lib().dto_checkout_tip_ff(self.h, ctypes.byref(out), ctypes.byref(ln), ctypes.byref(ff))
        if e:
            raise OracleError(e)
        data = ctypes.string_at(out.value, ln.value) if ln.value else b""
        lib().dto_free_buf(out)
        return data, bool(ff.value)

    def checkout_bytes(self, version, order=0) -> bytes:
        """ListOpLog::checkout(&[LV]) (src/list/oplog.rs:32-36) restated: walk Hist(version)."""
        v = (ctypes.c_int64 * max(1, len(version)))(*version)
        out = ctypes.c_void_p()
        ln = ctypes.c_size_t()
        st = Stats()
        e = lib().dto_checkout(self.h, v, len(version), order, ctypes.byref(out), ctypes.byref(ln), ctypes.byref(st))
        if e:
            raise OracleError(e)
        data = ctypes.string_at(out.value, ln.value) if ln.value else b""
        lib().dto_free_buf(out)
        return data

    def xf_operations(self):
        """(lv, xf) per LV in TransformedOpsIter order (xf -1: DeleteAlreadyHappened)."""
        n = len(self)
        buf = (ctypes.c_int64 * max(2, 2 * n))()
        e = lib().dto_xf_operations(self.h, buf)
        if e:
            raise OracleError(e)
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]

    def xf_operations_from(self, frm, merge):
        """(lv, xf) of iter_xf_operations_from(frm, merge) in TransformedOpsIter order."""
        n = len(self)
        buf = (ctypes.c_int64 * max(2, 2 * n))()
        a = (ctypes.c_int64 * max(1, len(frm)))(*frm)
        b = (ctypes.c_int64 * max(1, len(merge)))(*merge)
        k = ctypes.c_int64()
        e = lib().dto_xf_operations_from(self.h, a, len(frm), b, len(merge), buf, ctypes.byref(k))
        if e:
            raise OracleError(e)
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(k.value)]

    def checkout_tip(self, order=0) -> str:
        return self.checkout_tip_bytes(order).decode("utf-8")

    def stats(self):
        L = lib()
        return dict(lvs=len(self), agents=L.dto_num_agents(self.h), graph_entries=L.dto_num_graph_entries(self.h),
                    agent_runs=L.dto_num_agent_runs(self.h), ins_bytes=L.dto_ins_content_len(self.h))


def oplog_from_trace(txns, agent_name="jeremy"):
    """crates/bench/src/utils.rs:25-44 apply_edits_push_merge: per patch delete then insert."""
    o = OpLog()
    a = o.agent(agent_name)
    for txn in txns:
        for pos, dl, ins in txn["patches"]:
            if dl > 0:
                o.add_delete(a, pos, pos + dl)
            if ins:
                o.add_insert(a, pos, ins)
    return o


class Graph:
    def __init__(self, hist=()):
        self.h = lib().dto_graph_new()
        for e in hist:
            self.push(e["parents"], e["span"][0], e["span"][1])

    def __del__(self):
        if getattr(self, "h", None):
            lib().dto_graph_free(self.h)
            self.h = None

    def push(self, parents, start, end):
        a, n = _arr(parents)
        lib().dto_graph_push(self.h, a, n, start, end)

    def entries(self):
        L = lib()
        out = []
        s, e, sh = i64(), i64(), i64()
        for i in range(L.dto_graph_num_entries(self.h)):
            L.dto_graph_entry(self.h, i, ctypes.byref(s), ctypes.byref(e), ctypes.byref(sh))
            out.append((s.value, e.value, sh.value))
        return out

    def diff(self, a, b):
        A, na = _arr(a)
        B, nb = _arr(b)
        cap = 4 * lib().dto_graph_num_entries(self.h) + 64   # ranges <= 2 per entry
        oa = (ctypes.c_int64 * cap)()
        ob = (ctypes.c_int64 * cap)()
        ca, cb = ctypes.c_int(), ctypes.c_int()
        lib().dto_graph_diff(self.h, A, na, B, nb, oa, ctypes.byref(ca), ob, ctypes.byref(cb))
        return ([(oa[2 * i], oa[2 * i + 1]) for i in range(ca.value)],
                [(ob[2 * i], ob[2 * i + 1]) for i in range(cb.value)])

    def contains(self, frontier, target):
        A, n = _arr(frontier)
        return bool(lib().dto_graph_contains(self.h, A, n, target))

    def dominators(self, a, b=()):
        """find_dominators_2(a, b) / find_dominators(a): the union's members not in another
        member's history, ascending (dto_graph_dominators)."""
        A, na = _arr(a)
        B, nb = _arr(b)
        out = (ctypes.c_int64 * max(1, na + nb))()
        n = lib().dto_graph_dominators(self.h, A, na, B, nb, out)
        return list(out[:n])

    def find_conflicting(self, a, b):
        A, na = _arr(a)
        B, nb = _arr(b)
        spans = (ctypes.c_int64 * (6 * lib().dto_graph_num_entries(self.h) + 96))()
        common = (ctypes.c_int64 * 256)()   # OR_TP_M + 1 (dt_oracle.c)
        nc = ctypes.c_int()
        n = lib().dto_graph_find_conflicting(self.h, A, na, B, nb, spans, common, ctypes.byref(nc))
        flags = ["OnlyA", "OnlyB", "Shared"]
        return ([(spans[3 * i], spans[3 * i + 1], flags[spans[3 * i + 2]]) for i in range(n)],
                list(common[:nc.value]))
