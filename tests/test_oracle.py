"""Pin the CPU oracle against the reference's own fixtures before trusting it."""
import hashlib
import json
import os

import pytest

from oracle.oracle import Graph, OpLog, OracleError, oplog_from_trace, lib
import golden_data as G


# ---- 1/2. endContent goldens --------------------------------------------------------------
def test_friendsforever_dt_matches_flat_endcontent():
    # friendsforever_flat.json.gz is `dt export-trace-simple` of friendsforever.dt whose
    # end_content = oplog.checkout_tip() (crates/dt-cli/src/export.rs:233).
    o = OpLog.load_from(G.dt_bytes("friendsforever"))
    assert len(o) == 26078
    want = G.trace("friendsforever_flat")["endContent"]
    assert o.checkout_tip(order=0) == want
    assert o.checkout_tip(order=1) == want          # second topological order converges


@pytest.mark.parametrize("name", G.JSON_TRACES)
def test_json_trace_endcontent(name):
    # crates/bench/src/utils.rs:25-44 apply_edits_push_merge then checkout_tip
    t = G.trace(name)
    o = oplog_from_trace(t["txns"])
    assert o.checkout_tip() == t["endContent"]


@pytest.mark.parametrize("name", G.JSON_TRACES)
def test_json_trace_fast_forward_path(name):
    # the reference's FF path for linear histories (merge.rs:811-840), the CPU baseline of
    # BASELINE configs[0]: same text as the tracker and as endContent
    t = G.trace(name)
    o = oplog_from_trace(t["txns"])
    text, ff = o.checkout_tip_ff_bytes()
    assert ff and text == t["endContent"].encode()


def test_fast_forward_declines_concurrent_history():
    o = OpLog.load_from(G.dt_bytes("friendsforever"))
    text, ff = o.checkout_tip_ff_bytes()
    assert not ff and text == o.checkout_tip_bytes()


# ---- 3/4. compat byte vectors ------------------------------------------------------------
@pytest.mark.parametrize("vec", [G.COMPAT_SIMPLE_1, G.COMPAT_SIMPLE_2, G.COMPAT_SIMPLE_LZ4])
def test_compat_simple_doc(vec):
    o = OpLog.load_from(vec)
    assert len(o) == 8 + 4 + 1
    assert o.checkout_tip() == G.COMPAT_SIMPLE_TEXT
    assert o.frontier() == [12]


@pytest.mark.parametrize("vec", [G.COMPAT_EMPTY_1, G.COMPAT_EMPTY_2])
def test_compat_empty_doc(vec):
    o = OpLog.load_from(vec)
    assert len(o) == 0
    assert o.checkout_tip() == ""
    assert o.frontier() == []


def test_decode_vectors_from_reference_tests():
    vecs = json.load(open(os.path.join(G.HERE, "golden", "decode_vectors.json")))
    o = OpLog.load_from(bytes(vecs["merge_when_parents_unsorted.data"]))
    o.checkout_tip()                                 # must not panic (tests.rs:336-343)
    OpLog.load_from(bytes(vecs["regression_1.doc_data"]))


def test_crc_corruption_detected():
    # error_unrolling (tests.rs:180-235): flipping bytes must fail the CRC or decode cleanly.
    base = bytearray(G.COMPAT_SIMPLE_LZ4)
    ok = 0
    for i in range(len(base)):
        b = bytearray(base)
        b[i] ^= 0xFF
        try:
            o = OpLog.load_from(bytes(b))
            ok += 1
            o.checkout_tip()
        except OracleError:
            pass
    assert ok < len(base) // 4


def test_crc32c_known_answer():
    assert lib().dto_crc32c(b"123456789", 9) == 0xE3069283      # CRC-32/ISCSI check value


# ---- 5. causal_graph fixtures ------------------------------------------------------------
def _ranges(xs):
    return [tuple(x) if isinstance(x, list) else (x["start"], x["end"]) for x in xs]


@pytest.mark.parametrize("case", G.cg_fixture("diff"))
def test_cg_diff(case):
    g = Graph(case["hist"])
    a, b = g.diff(case["a"], case["b"])
    # fixture stores Graph::diff_slow output (descending spans, tools.rs:884-885)
    assert list(reversed(a)) == _ranges(case["expect_a"])
    assert list(reversed(b)) == _ranges(case["expect_b"])


@pytest.mark.parametrize("case", G.cg_fixture("version_contains"))
def test_cg_version_contains(case):
    g = Graph(case["hist"])
    assert g.contains(case["frontier"], case["target"]) == case["expected"]


@pytest.mark.parametrize("case", G.cg_fixture("conflicting"))
def test_cg_conflicting(case):
    g = Graph(case["hist"])
    spans, common = g.find_conflicting(case["a"], case["b"])
    want = [(s["start"], s["end"], f) for s, f in reversed(case["expect_spans"])]
    assert spans == want
    assert common == case["expect_common"]


def test_fancy_graph_shadows():
    # tools.rs:903-919
    g = Graph([{"span": [0, 3], "parents": []}, {"span": [3, 6], "parents": []},
               {"span": [6, 9], "parents": [1, 4]}, {"span": [9, 11], "parents": [2, 8]}])
    assert [e[2] for e in g.entries()] == [0, 3, 6, 6]



FANCY = [{"span": [0, 3], "parents": []}, {"span": [3, 6], "parents": []},
         {"span": [6, 9], "parents": [1, 4]}, {"span": [9, 11], "parents": [2, 8]}]
# dominator_smoke_test (tools.rs:1030-1051): (input, expected dominators)
DOMINATOR_KATS = [([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10], [5, 10]), ([10], [10]), ([5, 6], [5, 6]), ([5, 9], [5, 9]),
                  ([4, 9], [9]), ([1, 2], [2]), ([0, 2], [2]), ([0, 10], [10]), ([], []), ([2], [2]),
                  ([1, 4], [1, 4]), ([9, 10], [10]), ([2, 8, 9], [9]), ([2, 7, 9], [9]), ([6, 7], [7]), ([0], [0])]


@pytest.mark.parametrize("inp,want", DOMINATOR_KATS)
def test_dominator_kats(inp, want):
    """find_dominators of the input, and find_dominators_2 of every split of it into two
    dominator sets, both orders (check_dominators, tools.rs:993-1028)."""
    g = Graph(FANCY)
    assert g.dominators(inp) == want
    for k in range(len(inp) + 1):
        a, b = g.dominators(inp[:k]), g.dominators(inp[k:])
        assert g.dominators(a, b) == want and g.dominators(b, a) == want
    assert g.dominators([1, 1, 1]) == [1]   # dominator_duplicates (tools.rs:1053-1064)

# ---- 6. merge KATs (src/listmerge/merge.rs:1109-1325, src/list/branch.rs:166-193) ----------
def test_ff_merge_kat():
    o = OpLog()
    a, b = o.agent("a"), o.agent("b")
    o.add_insert_at(a, [], 0, "aaa")
    o.add_insert_at(b, [], 0, "bbb")
    assert o.checkout_tip() == "aaabbb"
    o.add_insert_at(a, [2, 5], 0, "ccc")
    assert o.checkout_tip() == "cccaaabbb"


def test_merge_inserts_name_tiebreak():
    o = OpLog()
    b, a = o.agent("b"), o.agent("a")          # agent ids in the other order: names decide
    o.add_insert_at(b, [], 0, "bbb")
    o.add_insert_at(a, [], 0, "aaa")
    assert o.checkout_tip() == "aaabbb"


@pytest.mark.parametrize("variant", [1, 2])
def test_merge_deletes(variant):
    o = OpLog()
    a, b = o.agent("a"), o.agent("b")
    t = o.add_insert(a, 0, "aaa")
    o.add_delete_at(a, [t], 1, 2)
    o.add_delete_at(b, [t], 0, 3)
    assert o.checkout_tip() == ""


def test_unroll_delete_text():
    o = OpLog()
    a = o.agent("a")
    o.add_insert(a, 0, "hi there")
    o.add_delete(a, 2, 5)
    assert o.checkout_tip() == "hiere"


def test_backspace_and_ins_back():
    o = OpLog()
    s = o.agent("seph")
    o.add_insert(s, 0, "abc")
    o.add_delete(s, 2, 3)
    o.add_delete(s, 1, 2)
    assert o.add_delete(s, 0, 1) == 5
    assert o.checkout_tip() == ""
    o2 = OpLog()
    s = o2.agent("seph")
    for c in "cba":
        o2.add_insert(s, 0, c)
    assert o2.checkout_tip() == "abc"


def test_branch_checkout_kat():
    # src/list/branch.rs:166-193 style: "hi there" then delete -> "hi"
    o = OpLog()
    s = o.agent("seph")
    o.add_insert(s, 0, "hi there")
    o.add_delete(s, 2, 8)
    assert o.checkout_tip() == "hi"


def test_unicode_content():
    o = OpLog()
    s = o.agent("seph")
    o.add_insert(s, 0, "héllo 𝄞 wörld")
    o.add_delete(s, 1, 2)
    o.add_insert(s, 6, "✓")
    assert o.checkout_tip() == "hllo 𝄞✓ wörld"
    text, ff = o.checkout_tip_ff_bytes()
    assert ff and text == "hllo 𝄞✓ wörld".encode()


# ---- 7. unpinned large docs: oracle-pinned by two-order convergence --------------------------
ORACLE_PINNED = {
    # sha256 prefix of the oracle's checkout (oracle-pinned, NOT reference-pinned)
    "git-makefile": (113676, "e9be745d89f8ce1f"),
    "node_nodecc": (38142, "c822bf881ad1fb04"),
}


@pytest.mark.parametrize("name", ["git-makefile", "node_nodecc"])
def test_large_docs_two_order_convergence(name):
    o = OpLog.load_from(G.dt_bytes(name))
    t0 = o.checkout_tip_bytes(order=0)
    n, h = ORACLE_PINNED[name]
    assert (len(t0), hashlib.sha256(t0).hexdigest()[:16]) == (n, h)
    if name == "node_nodecc":
        assert o.checkout_tip_bytes(order=1) == t0
