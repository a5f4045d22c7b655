"""Synthetic concurrent documents (dt_synth.cpp, BASELINE.json configs[3]): determinism, validity
against the CPU oracle, and host-side agreement.  GPU parity is in test_gpu_parity.py."""
import pytest

import dt_amd
from oracle.oracle import OpLog as OracleOpLog


def oracle_from_synth(doc, target=5000):
    na, ops = dt_amd.synth_ops(doc, target)
    o = OracleOpLog()
    ag = [o.agent(f"a{a}") for a in range(na)]
    for agent, kind, pos, ln, text, parents in ops:
        if kind == 0:
            o.add_insert_at(ag[agent], parents, pos, text)
        else:
            o.add_delete_at(ag[agent], parents, pos, pos + ln)
    return na, ops, o


def test_deterministic_and_sized():
    a = dt_amd.synth_ops(7, 5000)
    b = dt_amd.synth_ops(7, 5000)
    assert a == b
    na, ops = a
    assert 4 <= na <= 16
    n_lv = sum(op[3] for op in ops)
    assert 5000 <= n_lv < 5200
    assert dt_amd.synth_ops(8, 5000) != a


@pytest.mark.parametrize("doc", [0, 1, 2, 3, 17, 123456])
def test_oracle_accepts_synthetic_history(doc):
    """Every op position is valid in its agent's branch: the oracle (which checks bounds the way
    the reference panics, merge.rs:384,489) checks the whole history out."""
    na, ops, o = oracle_from_synth(doc, 2000)
    g = dt_amd.synth_oplog(doc, 2000)
    assert len(o) == len(g) == sum(op[3] for op in ops)
    assert g.local_frontier() == o.frontier()
    text = o.checkout_tip()
    assert text == o.checkout_tip(order=1)   # convergence across two topological orders
    # concurrency: the history has merges (entries with >= 2 parents)
    assert any(len(op[5]) >= 2 for op in ops)


def test_plan_matches_oracle_walk_on_synthetic():
    for doc in (0, 5, 9):
        _, _, o = oracle_from_synth(doc, 3000)
        g = dt_amd.synth_oplog(doc, 3000)
        ps = g.plan_stats()
        _, st = o.checkout_tip_bytes(order=0, with_stats=True)
        assert (ps["steps"], ps["retreat"], ps["advance"]) == (st["n_steps"], st["n_retreat"], st["n_advance"])
