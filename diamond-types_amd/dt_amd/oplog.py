"""The multi-CRDT `OpLog` (src/oplog.rs) as far as text checkout needs it.

One causal graph is shared by every CRDT of the document: map sets (`local_map_set` /
`remote_map_set`, oplog.rs:228-318) create child CRDTs (maps, registers, texts), text ops
(`local_text_op` / `remote_text_op`, :320-357) belong to one text CRDT.  `checkout_text(crdt)`
(:388-394) is `TextInfo::merge_into` (src/listmerge/merge.rs:954-1054): the text's ops with the
causal graph projected onto them (`Graph::subgraph_raw`, src/causalgraph/graph/subgraph.rs:39-250),
checked out by the list merge -- here `ListOpLog.project` (dtgpu_oplog_project) and the device
checkout.

Layout: every LV of the shared graph is an op of one `ListOpLog` (`self.log`); a map set occupies
its LV as a one-char placeholder insert (never part of a text's projection), a text op is the
text op itself.  `self.texts[crdt]` lists the text's LV spans (TextInfo.ops), `self.map_keys`
holds the map registers (MapInfo / RegisterInfo: every set, and the supremum of concurrent ones).

`ops_since` / `merge_ops` (oplog.rs:489-611) exchange changes as the `.dt` encoding of the shared
graph's ops after a version (`encode_from`, merged with `decode_and_add`, which skips what the
receiver has) plus the map / text ownership of each op keyed by its remote id (agent name, seq),
so two replicas converge whatever the merge order.
"""
from . import ListBranch, ListOpLog

ROOT_CRDT_ID = (1 << 64) - 1   # usize::MAX (src/lib.rs:332)
_PLACEHOLDER = "\x00"           # a map set's LV in the shared list

TEXT, MAP, REGISTER = "Text", "Map", "Register"


class NewCRDT:
    """CreateValue::NewCRDT(kind) (src/lib.rs)."""
    def __init__(self, kind):
        assert kind in (TEXT, MAP, REGISTER)
        self.kind = kind

    def __eq__(self, other):
        return isinstance(other, NewCRDT) and other.kind == self.kind

    def __repr__(self):
        return f"NewCRDT({self.kind})"


class OpLog:
    def __init__(self):
        self.log = ListOpLog()
        self.texts = {}        # text crdt LV -> [(start, end)] of its ops
        self.kinds = {ROOT_CRDT_ID: MAP}
        self.map_keys = {}     # (crdt, key) -> {"ops": [(lv, value)], "supremum": [index]}
        self.owner = {}        # run start LV -> ("map", crdt, key, value) | ("text", crdt, length)

    # ---- causal graph ---------------------------------------------------------------------------
    def get_or_create_agent_id(self, name: str) -> int:
        return self.log.get_or_create_agent_id(name)

    def version(self):
        return self.log.local_frontier()

    def __len__(self):
        return len(self.log)

    def _names(self):
        return self.log.export("agent_names")

    def _agent_of_name(self, name):
        names = self._names()
        for a, n in enumerate(names):
            if n == name:
                return a
        raise KeyError(name)

    def remote_id(self, lv):
        """LV -> (agent name, seq) (AgentAssignment::local_to_agent_version; a binary search in
        the native agent runs, dtgpu_oplog_local_to_remote)."""
        if lv == ROOT_CRDT_ID:
            return ("ROOT", 0)
        if not 0 <= lv < len(self.log):
            raise KeyError(lv)
        a, q = self.log.local_to_remote(lv)
        return (self._names()[a], q)

    def local_id(self, rid):
        if rid == ("ROOT", 0):
            return ROOT_CRDT_ID
        name, seq = rid
        return self.log.remote_to_local(self._agent_of_name(name), seq, 1)[0][0]

    # ---- maps ------------------------------------------------------------------------------------
    def _create(self, v, value):
        if isinstance(value, NewCRDT):
            self.kinds[v] = value.kind
            if value.kind == TEXT:
                self.texts.setdefault(v, [])

    def _set(self, crdt, key, v, value, remote):
        if crdt not in self.kinds or self.kinds[crdt] != MAP:
            raise KeyError(f"no map CRDT at {crdt}")
        self._create(v, value)
        reg = self.map_keys.setdefault((crdt, key), {"ops": [], "supremum": []})
        reg["ops"].append((v, value))
        if not remote:   # a local set dominates every earlier one (oplog.rs:234-256)
            reg["supremum"] = [len(reg["ops"]) - 1]
        else:            # the new supremum: the sets no other set of the register has seen
            lvs = [reg["ops"][i][0] for i in reg["supremum"]] + [v]
            dom = set(self.log.dominators(sorted(lvs)))
            reg["supremum"] = [i for i, (lv, _) in enumerate(reg["ops"]) if lv in dom]
        self.owner[v] = ("map", crdt, key, value)

    def local_map_set(self, agent: int, crdt: int, key: str, value) -> int:
        v = self.log.add_insert(agent, 0, _PLACEHOLDER)
        self._set(crdt, key, v, value, remote=False)
        return v

    def remote_map_set(self, agent: int, parents, crdt: int, key: str, value) -> int:
        v = self.log.add_insert_at(agent, parents, 0, _PLACEHOLDER)
        self._set(crdt, key, v, value, remote=True)
        return v

    def _tie_break(self, reg):
        """OpLog::tie_break_mv (oplog.rs:361-379): the supremum's winner by agent version order
        (AgentAssignment::tie_break_agent_versions: agent name, then seq)."""
        sup = reg["supremum"]
        if len(sup) == 1:
            return sup[0]
        return max(sup, key=lambda i: self.remote_id(reg["ops"][i][0]))

    def map_get(self, crdt, key):
        reg = self.map_keys.get((crdt, key))
        if not reg or not reg["supremum"]:
            return None
        lv, value = reg["ops"][self._tie_break(reg)]
        return (lv, value)

    def crdt_at_path(self, path):
        """OpLog::crdt_at_path (oplog.rs:428-454): (kind, crdt LV)."""
        kind, crdt = MAP, ROOT_CRDT_ID
        for k in path:
            if kind != MAP:
                raise KeyError(path)
            got = self.map_get(crdt, k)
            if got is None or not isinstance(got[1], NewCRDT):
                raise KeyError(path)
            crdt, kind = got[0], got[1].kind
        return kind, crdt

    def text_at_path(self, path):
        kind, crdt = self.crdt_at_path(path)
        if kind != TEXT:
            raise KeyError(path)
        return crdt

    # ---- texts -----------------------------------------------------------------------------------
    def _text(self, crdt):
        if self.kinds.get(crdt) != TEXT:
            raise KeyError(f"no text CRDT at {crdt}")
        return self.texts[crdt]

    def _push(self, crdt, start, end):
        spans = self._text(crdt)
        if spans and spans[-1][1] == start:
            spans[-1] = (spans[-1][0], end)
        else:
            spans.append((start, end))
        self.owner[start] = ("text", crdt, end - start)

    def local_spans(self, rid, n):
        """Local LV spans of the remote ids (name, seq .. seq + n), in seq order
        (dtgpu_oplog_remote_to_local: a binary search in the agent's seq runs)."""
        name, seq = rid
        return [(int(b), int(e)) for b, e in self.log.remote_to_local(self._agent_of_name(name), seq, n)]

    def local_text_op(self, agent: int, crdt: int, op):
        """op: ("ins", pos, content) or ("del", start, end) (TextOperation::new_insert /
        new_delete).  Returns the op's LV span."""
        self._text(crdt)
        n0 = len(self.log)
        if op[0] == "ins":
            self.log.add_insert(agent, op[1], op[2])
        else:
            self.log.add_delete_without_content(agent, op[1], op[2])
        self._push(crdt, n0, len(self.log))
        return (n0, len(self.log))

    def remote_text_op(self, agent: int, parents, crdt: int, op):
        self._text(crdt)
        n0 = len(self.log)
        if op[0] == "ins":
            self.log.add_insert_at(agent, parents, op[1], op[2])
        else:
            self.log.add_delete_at(agent, parents, op[1], op[2])
        self._push(crdt, n0, len(self.log))
        return (n0, len(self.log))

    def checkout_text_bytes(self, crdt: int) -> bytes:
        """OpLog::checkout_text (oplog.rs:388-394): the text's projected ops checked out on the
        device (an empty text has no ops to project)."""
        spans = self._text(crdt)
        if not spans:
            return b""
        return self.log.project(spans).checkout_tip_bytes()

    def checkout_text(self, crdt: int) -> str:
        return self.checkout_text_bytes(crdt).decode()

    def merge_text_into(self, crdt: int, content: str, frm, merge_frontier=None) -> str:
        """TextInfo::merge_into(into, cg, from, merge_frontier) (src/listmerge/merge.rs:1022-1054,
        via with_xf_iter :954-985): the text's ops with the shared graph projected onto them
        (dtgpu_oplog_project), `from` and `merge_frontier` projected the same way
        (project_onto_subgraph_raw), and the transformed operations between the two -- replayed
        on the device (dtgpu_xf_operations_from, f1) -- applied to `content`, the text as the
        branch holds it at `from`."""
        spans = self._text(crdt)
        if merge_frontier is None:
            merge_frontier = self.version()
        if not spans:
            return content
        sub = self.log.project(spans)
        pf = self.log.project_version(spans, list(frm))
        pm = self.log.project_version(spans, list(merge_frontier))
        b = ListBranch(content.encode(), pf)
        b.merge(sub, pm)
        return b.content()

    def checkout(self, crdt=ROOT_CRDT_ID):
        """OpLog::checkout / checkout_map (oplog.rs:396-426): registers resolved, child maps and
        texts checked out."""
        out = {}
        for (c, key), reg in sorted(self.map_keys.items(), key=lambda kv: kv[0][1]):
            if c != crdt or not reg["supremum"]:
                continue
            lv, value = reg["ops"][self._tie_break(reg)]
            if isinstance(value, NewCRDT):
                out[key] = self.checkout_text(lv) if value.kind == TEXT else (
                    self.checkout(lv) if value.kind == MAP else None)
            else:
                out[key] = value
        return out

    # ---- exchange ----------------------------------------------------------------------------------
    def ops_since(self, since=()):
        """OpLog::ops_since (oplog.rs:489-566): the shared graph's ops after `since` as a `.dt`
        patch, with each op run's owner keyed by remote id."""
        data = self.log.encode_from(list(since))
        meta = []
        for lv, own in sorted(self.owner.items()):
            rid = self.remote_id(lv)
            if own[0] == "map":
                _, crdt, key, value = own
                meta.append(("map", rid, self.remote_id(crdt), key, value))
            else:
                meta.append(("text", rid, self.remote_id(own[1]), own[2]))
        return data, meta

    def merge_ops(self, changes):
        """OpLog::merge_ops (oplog.rs:568-611): add the patch (ops already here are skipped) and
        adopt the ownership of the ops that were new."""
        data, meta = changes
        known = len(self.log)
        self.log.decode_and_add(data)
        for rec in meta:
            if rec[0] == "map":
                _, rid, crdt_rid, key, value = rec
                lv = self.local_id(rid)
                if lv >= known:   # new here (decode_and_add skipped what was known)
                    self._set(self.local_id(crdt_rid), key, lv, value, remote=True)
            else:
                _, rid, crdt_rid, n = rec
                crdt = self.local_id(crdt_rid)
                for b, e in self.local_spans(rid, n):
                    if b >= known:
                        self._push(crdt, b, e)
        for crdt, spans in self.texts.items():   # spans in LV order, adjacent ones joined
            spans.sort()
            merged = []
            for b, e in spans:
                if merged and merged[-1][1] == b:
                    merged[-1] = (merged[-1][0], e)
                else:
                    merged.append((b, e))
            self.texts[crdt] = merged


class Branch:
    """`Branch` (src/branch.rs): a checkout of every CRDT of an `OpLog` at `frontier`.  Texts are
    kept as strings and moved forward with TextInfo::merge_into (branch.rs:180-232,
    merge_changes_to_tip); registers and maps are resolved from the oplog at the branch's version
    (only the tip is supported for them, as merge_changes_to_tip moves the branch there)."""

    def __init__(self):
        self.frontier = []
        self.texts = {}

    def merge_changes_to_tip(self, oplog: OpLog) -> None:
        """Branch::merge_changes_to_tip (branch.rs:180-232): every text CRDT's new ops are merged
        into this branch's copy of it, from the branch's frontier to the oplog's tip."""
        tip = oplog.version()
        for crdt, spans in oplog.texts.items():
            if not spans:
                self.texts.setdefault(crdt, "")
                continue
            self.texts[crdt] = oplog.merge_text_into(crdt, self.texts.get(crdt, ""), self.frontier, tip)
        self.frontier = list(tip)

    def text(self, crdt: int) -> str:
        return self.texts.get(crdt, "")
