"""The multi-CRDT OpLog mirror (dt_amd/oplog.py, src/oplog.rs): map sets creating text CRDTs on
one shared causal graph, text ops per CRDT, checkout_text through the subgraph projection and
the device checkout; ops_since / merge_ops convergence.

Pinned by the reference's own oplog tests (src/oplog.rs:640-704: `text` -> "hai!", and
`concurrent_changes`) and, for concurrent edits of one text interleaved with other CRDTs'
ops, by the C oracle's checkout of the same text ops as a plain list oplog (the projection
must drop every foreign LV and keep the text's causal order)."""
import random

import pytest

import dt_amd
from dt_amd.oplog import MAP, ROOT_CRDT_ID, TEXT, Branch, NewCRDT, OpLog
from oracle.oracle import OpLog as OracleOpLog


def _text_doc():
    o = OpLog()
    seph = o.get_or_create_agent_id("seph")
    text = o.local_map_set(seph, ROOT_CRDT_ID, "content", NewCRDT(TEXT))
    o.local_text_op(seph, text, ("ins", 0, "Oh hai!"))
    o.local_text_op(seph, text, ("del", 0, 3))
    title = o.local_map_set(seph, ROOT_CRDT_ID, "title", NewCRDT(TEXT))
    o.local_text_op(seph, title, ("ins", 0, "Please read this cool info"))
    return o, text, title


def test_structure_of_the_reference_text_test():
    """oplog.rs:641-657: two texts under the root map, one LV per map set."""
    o, text, title = _text_doc()
    assert len(o) == 1 + 7 + 3 + 1 + 26
    assert o.texts[text] == [(1, 11)] and o.texts[title] == [(12, 38)]
    assert o.crdt_at_path(["content"]) == (TEXT, text)
    assert o.text_at_path(["title"]) == title
    with pytest.raises(KeyError):
        o.text_at_path(["nope"])
    # the projection keeps only the text's own ops, in a chain
    sub = o.log.project(o.texts[text])
    assert len(sub) == 10 and sub.local_frontier() == [9]


def test_merge_ops_roundtrip_structure():
    o, text, title = _text_doc()
    o2 = OpLog()
    o2.merge_ops(o.ops_since([]))
    assert o2.texts == o.texts and o2.kinds == o.kinds
    assert o2.map_keys.keys() == o.map_keys.keys()
    # merging the same changes again adds nothing
    o2.merge_ops(o.ops_since([]))
    assert o2.texts == o.texts and len(o2) == len(o)


def test_concurrent_map_sets_keep_both_in_the_supremum():
    a, b = OpLog(), OpLog()
    x, y = a.get_or_create_agent_id("a"), b.get_or_create_agent_id("b")
    a.local_map_set(x, ROOT_CRDT_ID, "k", 1)
    b.local_map_set(y, ROOT_CRDT_ID, "k", 2)
    a.merge_ops(b.ops_since([]))
    b.merge_ops(a.ops_since([]))
    for o in (a, b):
        reg = o.map_keys[(ROOT_CRDT_ID, "k")]
        assert len(reg["supremum"]) == 2
        assert o.map_get(ROOT_CRDT_ID, "k")[1] == 2   # tie-break: agent "b" > "a"


@pytest.mark.gpu
def test_gpu_reference_text_kat():
    """src/oplog.rs:654: checkout_text(text) == "hai!"."""
    o, text, title = _text_doc()
    assert o.checkout_text(text) == "hai!"
    assert o.checkout_text(title) == "Please read this cool info"
    assert o.checkout() == {"content": "hai!", "title": "Please read this cool info"}


@pytest.mark.gpu
def test_gpu_concurrent_changes_converge():
    """src/oplog.rs:675-704: two replicas, one text each, merged both ways: same checkout."""
    o1, o2 = OpLog(), OpLog()
    seph = o1.get_or_create_agent_id("seph")
    text = o1.local_map_set(seph, ROOT_CRDT_ID, "content", NewCRDT(TEXT))
    o1.local_text_op(seph, text, ("ins", 0, "Oh hai!"))
    kaarina = o2.get_or_create_agent_id("kaarina")
    title = o2.local_map_set(kaarina, ROOT_CRDT_ID, "title", NewCRDT(TEXT))
    o2.local_text_op(kaarina, title, ("ins", 0, "Better keep it clean"))
    o2.merge_ops(o1.ops_since([]))
    o1.merge_ops(o2.ops_since([]))
    assert o1.checkout() == o2.checkout() == {"content": "Oh hai!", "title": "Better keep it clean"}
    assert o1.crdt_at_path(["title"])[0] == TEXT


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_concurrent_text_edits_match_oracle(seed):
    """Three agents edit one text concurrently (explicit parents), interleaved with map sets
    and a second text: checkout_text equals the oracle's checkout of the same text ops as a
    plain list oplog, and every replica built by merge_ops in another order agrees."""
    rng = random.Random(seed)
    o = OpLog()
    ag = [o.get_or_create_agent_id(n) for n in ("amy", "bob", "cat")]
    text = o.local_map_set(ag[0], ROOT_CRDT_ID, "body", NewCRDT(TEXT))
    other = o.local_map_set(ag[1], ROOT_CRDT_ID, "note", NewCRDT(TEXT))
    plain = OracleOpLog()
    pa = [plain.agent(n) for n in ("amy", "bob", "cat")]
    lv_map = {}                # shared-graph LV of a body op -> plain-oplog LV
    heads = [[] for _ in ag]   # each agent's version in the shared graph (body ops only)
    for step in range(40):
        i = rng.randrange(3)
        if rng.random() < 0.2:   # another CRDT's op, concurrent with everything
            o.local_map_set(ag[i], ROOT_CRDT_ID, f"k{step}", step)
            continue
        if rng.random() < 0.1:
            o.local_text_op(ag[i], other, ("ins", 0, "x"))
            continue
        if rng.random() < 0.25:   # merge another agent's view
            j = rng.randrange(3)
            heads[i] = o.log.dominators(sorted(set(heads[i]) | set(heads[j])))
        parents = heads[i]
        pv = sorted(lv_map[x] for x in parents)
        n = len(plain.checkout_bytes(pv).decode()) if pv else 0   # the text at this version
        n0 = len(o)
        if n > 2 and rng.random() < 0.35:
            s0 = rng.randrange(n - 1)
            e0 = min(n, s0 + rng.randint(1, 2))
            o.remote_text_op(ag[i], parents, text, ("del", s0, e0))
            plv = plain.add_delete_at(pa[i], pv, s0, e0)
        else:
            p = rng.randrange(n + 1)
            c = rng.choice(["ab", "c", "dé", "f"])
            o.remote_text_op(ag[i], parents, text, ("ins", p, c))
            plv = plain.add_insert_at(pa[i], pv, p, c)
        n1 = len(o)
        for k in range(n1 - n0):
            lv_map[n0 + k] = plv - (n1 - n0 - 1) + k
        heads[i] = [n1 - 1]
    want = plain.checkout_tip_bytes()
    assert o.checkout_text_bytes(text) == want
    r = OpLog()   # a replica built by merge_ops
    r.merge_ops(o.ops_since([]))
    assert r.checkout_text_bytes(text) == want


def test_native_remote_id_lookups():
    """remote_id / local_id / local_spans go through the native agent-run searches
    (dtgpu_oplog_local_to_remote / remote_to_local) and agree with a scan of the agent runs."""
    o = OpLog()
    ag = [o.get_or_create_agent_id(n) for n in ("amy", "bob")]
    text = o.local_map_set(ag[0], ROOT_CRDT_ID, "t", NewCRDT(TEXT))
    for k in range(30):
        o.local_text_op(ag[k % 2], text, ("ins", 0, "ab"[k % 2] * (1 + k % 3)))
    names = o._names()
    runs = o.log.export("agent_runs").reshape(-1, 4)
    for s0, n, a, q in runs:
        for k in range(int(n)):
            lv = int(s0) + k
            rid = (names[a], int(q) + k)
            assert o.remote_id(lv) == rid
            assert o.local_id(rid) == lv
    # a remote span crossing runs comes back in seq order
    name, q0 = o.remote_id(runs[1][0])
    spans = o.local_spans((name, q0), 3)
    assert sum(e - b for b, e in spans) == 3
    with pytest.raises(KeyError):
        o.local_id(("amy", 10_000))
    with pytest.raises(KeyError):
        o.local_id(("zed", 0))


def _random_text_history(seed, steps):
    """The generator of test_gpu_concurrent_text_edits_match_oracle, as a step function: each
    call adds one op (text, other CRDTs) and mirrors the text's ops into a plain oracle oplog."""
    rng = random.Random(seed)
    o = OpLog()
    ag = [o.get_or_create_agent_id(n) for n in ("amy", "bob", "cat")]
    text = o.local_map_set(ag[0], ROOT_CRDT_ID, "body", NewCRDT(TEXT))
    other = o.local_map_set(ag[1], ROOT_CRDT_ID, "note", NewCRDT(TEXT))
    plain = OracleOpLog()
    pa = [plain.agent(n) for n in ("amy", "bob", "cat")]
    lv_map = {}
    heads = [[] for _ in ag]

    def step(k):
        i = rng.randrange(3)
        if rng.random() < 0.2:
            o.local_map_set(ag[i], ROOT_CRDT_ID, f"k{k}", k)
            return
        if rng.random() < 0.1:
            o.local_text_op(ag[i], other, ("ins", 0, "x"))
            return
        if rng.random() < 0.25:
            j = rng.randrange(3)
            heads[i] = o.log.dominators(sorted(set(heads[i]) | set(heads[j])))
        parents = heads[i]
        pv = sorted(lv_map[x] for x in parents)
        n = len(plain.checkout_bytes(pv).decode()) if pv else 0
        n0 = len(o)
        if n > 2 and rng.random() < 0.35:
            s0 = rng.randrange(n - 1)
            e0 = min(n, s0 + rng.randint(1, 2))
            o.remote_text_op(ag[i], parents, text, ("del", s0, e0))
            plv = plain.add_delete_at(pa[i], pv, s0, e0)
        else:
            p = rng.randrange(n + 1)
            c = rng.choice(["ab", "c", "dé", "f"])
            o.remote_text_op(ag[i], parents, text, ("ins", p, c))
            plv = plain.add_insert_at(pa[i], pv, p, c)
        n1 = len(o)
        for q in range(n1 - n0):
            lv_map[n0 + q] = plv - (n1 - n0 - 1) + q
        heads[i] = [n1 - 1]

    return o, text, other, plain, lv_map, step


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_branch_merge_into_from_a_non_empty_version(seed):
    """TextInfo::merge_into from an existing branch version (src/listmerge/merge.rs:1022-1054, as
    Branch::merge_changes_to_tip calls it, src/branch.rs:223): a branch checked out part way
    through a concurrent history, then moved to the tip in one or two merges, holds the oracle's
    checkout of the same text ops; a merge at an older, concurrent version (the version one agent
    saw) too."""
    o, text, other, plain, lv_map, step = _random_text_history(seed, 60)
    for k in range(25):
        step(k)
    br = Branch()
    br.merge_changes_to_tip(o)
    mid_plain = plain.checkout_tip_bytes()
    assert br.text(text).encode() == mid_plain
    mid_version = list(br.frontier)
    for k in range(25, 45):
        step(k)
    br.merge_changes_to_tip(o)
    assert br.text(text).encode() == plain.checkout_tip_bytes()
    assert br.text(other) == o.checkout_text(other)
    for k in range(45, 60):
        step(k)
    br.merge_changes_to_tip(o)
    want = plain.checkout_tip_bytes()
    assert br.text(text).encode() == want
    # from the mid version straight to the tip
    assert o.merge_text_into(text, mid_plain.decode(), mid_version).encode() == want
    # from the mid version to mid + one agent's later head (a version concurrent with the tip):
    # the oracle's text at the same version, found through the projection (the text's ops in
    # LV order are the projected numbering; lv_map takes them to the plain oplog)
    text_lvs = sorted(lv_map)
    for head in sorted(lv_map)[-3:]:
        target = o.log.dominators(mid_version, [head])
        pf = o.log.project_version(o.texts[text], target)
        plain_v = sorted(lv_map[text_lvs[i]] for i in pf)   # the history of a set is the history of its frontier
        got = o.merge_text_into(text, mid_plain.decode(), mid_version, target)
        assert got.encode() == plain.checkout_bytes(plain_v)
