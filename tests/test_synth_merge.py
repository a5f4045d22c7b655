"""The SURVEY.md 8(d)4 synthetic generator (dt_synth.cpp MergeGen; BASELINE configs[3]):
per-step pairwise merges with p = 0.1 (find_dominators_2) over make_random_change edits.
CPU: determinism, shape (agents, LVs, partially merged graphs), two-order oracle convergence.
GPU (-m gpu): 64 generated documents plus wide ones (more causal chains than the device prep
takes) checked out on the device against the oracle -- device-staged where the device takes
them, DECODE_DEFER and a correct host-staged checkout where it does not."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, ROOT)
import dt_amd  # noqa: E402
from oracle.oracle import OpLog as OracleOpLog  # noqa: E402


def shape(o):
    ents = [tuple(e) for e in o.export("entries")]
    offs = list(o.export("parent_offsets"))
    merges = sum(1 for i in range(len(ents)) if offs[i + 1] - offs[i] >= 2)
    names = o.export("agent_names")
    return len(ents), merges, len(names)


def test_deterministic_and_shaped():
    a = dt_amd.synth_merge_oplog(3, 5000).encode()
    b = dt_amd.synth_merge_oplog(3, 5000).encode()
    assert a == b
    agents = set()
    for d in range(16):
        o = dt_amd.synth_merge_oplog(d, 5000)
        ne, merges, na = shape(o)
        assert 5000 <= len(o) < 5000 + 16
        assert 4 <= na <= 16
        agents.add(na)
        assert merges > 0 and ne > merges          # partially merged: merge entries among linear runs
        assert len(o.local_frontier()) >= 1
    assert len(agents) > 3


@pytest.mark.parametrize("doc", [0, 5, 11, 23])
def test_oracle_two_orders_agree(doc):
    o = OracleOpLog.load_from(dt_amd.synth_merge_oplog(doc, 4000).encode())
    assert o.checkout_tip_bytes(order=0) == o.checkout_tip_bytes(order=1)


def test_wide_variant_has_many_concurrent_heads():
    o = dt_amd.synth_merge_oplog(7, 5000, 96)
    assert len(o.export("agent_names")) == 96
    assert len(o.local_frontier()) > 64


def _pool():
    docs = [dt_amd.synth_merge_oplog(d, 5000).encode() for d in range(64)]
    wide = [dt_amd.synth_merge_oplog(1000 + d, 5000, 96).encode() for d in range(2)]
    return docs, wide


@pytest.mark.gpu
def test_gpu_device_staged_synth_merge_docs_match_oracle():
    docs, wide = _pool()
    allv = docs + wide
    b = dt_amd.Batch(docs=allv, staging="device")
    b.run()
    b.sync()
    res = b.results()
    deferred = []
    for i, d in enumerate(allv):
        want = OracleOpLog.load_from(d).checkout_tip_bytes()
        if res[i]["status"] == dt_amd.DECODE_DEFER:
            deferred.append(i)
            continue
        assert res[i]["status"] == 0, (i, res[i])
        assert b.text(i) == want, i
    # only the wide documents (96 agents: past the device prep's 64 causal chains) are handed
    # back; every ordinary 4-16-agent document checks out on the device path
    assert set(deferred) == set(range(len(docs), len(allv))), deferred
    # the documented retry: the host-staged batch checks the deferred ones out on the device
    h = dt_amd.Batch(docs=[allv[i] for i in deferred], staging="host")
    h.run()
    h.sync()
    for k, i in enumerate(deferred):
        assert h.results()[k]["status"] == 0
        assert h.text(k) == OracleOpLog.load_from(allv[i]).checkout_tip_bytes(), i


@pytest.mark.gpu
def test_gpu_host_staged_synth_merge_docs_match_oracle():
    docs, wide = _pool()
    oplogs = [dt_amd.synth_merge_oplog(d, 5000) for d in range(16)] + [dt_amd.synth_merge_oplog(1000, 5000, 96)]
    b = dt_amd.Batch(oplogs=oplogs)
    b.run()
    b.sync()
    for i, o in enumerate(oplogs):
        assert b.results()[i]["status"] == 0
        assert b.text(i) == OracleOpLog.load_from(o.encode()).checkout_tip_bytes(), i
