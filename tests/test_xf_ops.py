"""`ListOpLog::iter_xf_operations()` (src/list/merge.rs:24-48): the transformed operations in
`TransformedOpsIter` order (src/listmerge/merge.rs:788-940).

Golden: `friendsforever_flat.json.gz` is `dt export-trace-simple` of friendsforever.dt, whose
patches are exactly the reference's iter_xf_operations() stream (crates/dt-cli/src/export.rs:
188-238, split into txns at agent changes).  Streams are compared by effect: the inserts must
match one for one (position and char) and the document before every insert must be the same
(deletes are grouped differently -- the reference reports a backspace run as one range,
split at its content-tree entries).

CPU: the oracle's stream (tests/golden pinning of the oracle) and the engine's host application
order.  GPU: the device's per-LV transformed positions equal the oracle's exactly.
"""
import random

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, oplog_from_trace as oracle_from_trace
import dt_amd


def _per_char(oplog_exports, stream):
    """(lv, pos|None) stream -> [('I', pos, ch) | ('D', pos)] using the engine oplog's arrays."""
    ops, content, coff = oplog_exports
    kind = {}
    for lv, ln, _pos, kf in ops:
        for k in range(int(ln)):
            kind[int(lv) + k] = int(kf) & 1
    out = []
    for lv, x in stream:
        if x is None or x < 0:
            continue
        if kind[lv] == 0:
            b = int(coff[lv])
            out.append(("I", x, content[b:b + 4].decode("utf-8", errors="ignore")[:1]))
        else:
            out.append(("D", x))
    return out


def _exports(o):
    return o.export("ops").reshape(-1, 4), bytes(o.export("content")), o.export("char_offsets")


def _flat_per_char(trace):
    out = []
    for txn in trace["txns"]:
        for pos, d, ins in txn["patches"]:
            out.extend(("D", pos) for _ in range(d))
            out.extend(("I", pos + k, c) for k, c in enumerate(ins))
    return out


def _states(seq):
    """The inserts of a per-char stream, each with the document it applies to."""
    s, out = "", []
    for op in seq:
        if op[0] == "D":
            s = s[:op[1]] + s[op[1] + 1:]
        else:
            out.append((op[1], op[2], s))
            s = s[:op[1]] + op[2] + s[op[1]:]
    return out, s


def _assert_same_effect(mine, ref, end):
    a, sa = _states(mine)
    b, sb = _states(ref)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert x == y, f"insert {i}: {x[:2]} vs {y[:2]}"
    assert sa == sb == end


def test_oracle_xf_stream_matches_reference_export():
    data = G.dt_bytes("friendsforever")
    ora = OracleOpLog.load_from(data)
    eng = dt_amd.ListOpLog.load_from(data)
    t = G.trace("friendsforever_flat")
    mine = _per_char(_exports(eng), ora.xf_operations())
    ref = _flat_per_char(t)
    assert len(mine) == len(ref) == 26078
    _assert_same_effect(mine, ref, t["endContent"])


@pytest.mark.parametrize("name", G.DT_FILES)
def test_host_xf_order_matches_oracle(name):
    data = G.dt_bytes(name)
    order = dt_amd.ListOpLog.load_from(data).xf_order()
    assert order == [lv for lv, _ in OracleOpLog.load_from(data).xf_operations()]


def test_host_xf_order_synthetic():
    for doc in range(4):
        o = dt_amd.synth_oplog(doc, 2000)
        ora = _oracle_copy(o)
        assert o.xf_order() == [lv for lv, _ in ora.xf_operations()], doc
        assert sorted(o.xf_order()) == list(range(len(o)))


def _oracle_copy(o):
    from test_checkout_version import _oracle_rebuild
    return _oracle_rebuild(o)


def test_linear_trace_xf_is_identity():
    """A single-agent trace fast-forwards entirely: every op keeps its own position."""
    t = G.trace("sveltecomponent")
    ora = oracle_from_trace(t["txns"])
    xf = ora.xf_operations()
    eng = dt_amd.oplog_from_trace(t["txns"])
    ops = eng.export("ops").reshape(-1, 4)
    want = {}
    for lv, ln, pos, kf in ops:
        lv, ln, pos, kf = int(lv), int(ln), int(pos), int(kf)
        for k in range(ln):
            want[lv + k] = pos + k if kf & 1 == 0 else (pos if kf & 2 else pos + ln - 1 - k)
    assert [lv for lv, _ in xf] == list(range(len(eng)))
    assert all(x == want[lv] for lv, x in xf)


# ---- GPU ----------------------------------------------------------------------------------

@pytest.mark.gpu
def test_gpu_xf_matches_reference_export():
    data = G.dt_bytes("friendsforever")
    eng = dt_amd.ListOpLog.load_from(data)
    t = G.trace("friendsforever_flat")
    mine = _per_char(_exports(eng), eng.xf_operations_lv())
    _assert_same_effect(mine, _flat_per_char(t), t["endContent"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", G.DT_FILES)
def test_gpu_xf_matches_oracle(name):
    data = G.dt_bytes(name)
    got = dt_amd.ListOpLog.load_from(data).xf_operations_lv()
    want = [(lv, None if x < 0 else x) for lv, x in OracleOpLog.load_from(data).xf_operations()]
    assert len(got) == len(want)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, (len(bad), bad[0], got[bad[0]], want[bad[0]])


@pytest.mark.gpu
def test_gpu_xf_synthetic_and_kats():
    rng = random.Random(1)
    for doc in rng.sample(range(1000), 4):
        o = dt_amd.synth_oplog(doc, 3000)
        want = [(lv, None if x < 0 else x) for lv, x in _oracle_copy(o).xf_operations()]
        assert o.xf_operations_lv() == want, doc
    for vec in (G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_LZ4):
        o = dt_amd.ListOpLog.load_from(vec)
        want = [(lv, None if x < 0 else x) for lv, x in OracleOpLog.load_from(vec).xf_operations()]
        assert o.xf_operations_lv() == want


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_gpu_iter_xf_operations_rebuild_the_text(name):
    """Applying the merged (range, op) stream to an empty document gives checkout_tip()."""
    o = dt_amd.ListOpLog.load_from(G.dt_bytes(name))
    s = []
    n = 0
    for rng, op in o.iter_xf_operations():
        n += len(rng)
        if op is None:
            continue
        if op[0] == "ins":
            s[op[1]:op[1]] = list(op[2])
        else:
            del s[op[1]:op[1] + op[2]]
    assert n == len(o)
    assert "".join(s) == o.checkout_tip().content()


# ---- incremental merges: iter_xf_operations_from / ListBranch::merge ------------------------

def _pairs(o, rng, k):
    n = len(o)
    out = []
    for _ in range(k):
        a = o.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2]))))
        b = o.dominators(sorted(rng.sample(range(n), rng.choice([1, 1, 2]))))
        out.append((a, b))
    out.append(([], o.local_frontier()))
    out.append((o.local_frontier(), o.local_frontier()))
    return out


def _apply(text, ops):
    s = text
    for op in ops:
        s = s[:op[1]] + s[op[1] + 1:] if op[0] == "D" else s[:op[1]] + op[2] + s[op[1]:]
    return s


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_oracle_xf_from_rebuilds_the_merged_checkout(name):
    """The oracle's incremental stream, applied to the checkout at `from`, gives the checkout at
    find_dominators_2(from, merging) -- the invariant ListBranch::merge relies on."""
    data = G.dt_bytes(name)
    ora = OracleOpLog.load_from(data)
    eng = dt_amd.ListOpLog.load_from(data)
    ex = _exports(eng)
    for a, b in _pairs(eng, random.Random(21), 8 if name == "friendsforever" else 1):
        got = _apply(ora.checkout_bytes(a).decode(), _per_char(ex, ora.xf_operations_from(a, b)))
        assert got == ora.checkout_bytes(eng.dominators(a, b)).decode(), (a, b)


@pytest.mark.parametrize("name", ["friendsforever", "git-makefile", "node_nodecc"])
def test_host_xf_from_order_matches_oracle(name):
    data = G.dt_bytes(name)
    ora = OracleOpLog.load_from(data)
    eng = dt_amd.ListOpLog.load_from(data)
    for a, b in _pairs(eng, random.Random(5), 6 if name == "friendsforever" else 1):
        assert eng.xf_order(a, b) == [lv for lv, _ in ora.xf_operations_from(a, b)], (a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["friendsforever", "git-makefile"])
def test_gpu_xf_from_matches_oracle(name):
    data = G.dt_bytes(name)
    ora = OracleOpLog.load_from(data)
    eng = dt_amd.ListOpLog.load_from(data)
    for a, b in _pairs(eng, random.Random(17), 6 if name == "friendsforever" else 2):
        want = [(lv, None if x < 0 else x) for lv, x in ora.xf_operations_from(a, b)]
        assert eng.xf_operations_lv(a, b) == want, (a, b)


@pytest.mark.gpu
def test_gpu_branch_merge_applies_transformed_ops():
    """ListBranch::merge chains (src/list/merge.rs:63-95): every step's content equals the
    oracle's checkout at the branch's new version; the last merge reaches the golden text."""
    data = G.dt_bytes("friendsforever")
    ora = OracleOpLog.load_from(data)
    o = dt_amd.ListOpLog.load_from(data)
    rng = random.Random(29)
    br = dt_amd.ListBranch.new()
    for _ in range(5):
        br.merge(o, [rng.randrange(len(o))])
        assert br.content_bytes() == ora.checkout_bytes(br.local_frontier())
    br.merge(o, o.local_frontier())
    assert br.content() == G.trace("friendsforever_flat")["endContent"]
    for doc in range(2):
        s = dt_amd.synth_oplog(doc, 2000)
        sora = _oracle_copy(s)
        br = dt_amd.ListBranch.new_at_local_version(s, [len(s) // 3])
        br.merge(s, [2 * len(s) // 3])
        assert br.content_bytes() == sora.checkout_bytes(br.local_frontier())
