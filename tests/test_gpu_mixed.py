"""BASELINE configs[4]: one device-staged, skewed batch of all 8 benchmark_data traces (3 .dt
files + the 5 JSON traces written as .dt the way crates/bench/src/utils.rs:25-44 builds their
oplogs, written by the native encoder), ~36x apart in LVs, every document checked against its golden endContent (the JSON
traces, friendsforever) or the oracle (git-makefile, node_nodecc: oracle-pinned)."""
import gzip
import json
import os

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def mixed():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")
    docs, want = [], []
    for n in G.DT_FILES:
        d = G.dt_bytes(n)
        docs.append(d)
        if n == "friendsforever":
            want.append(json.load(gzip.open(os.path.join(ROOT, "tests", "golden", "benchmark_data",
                                                          "friendsforever_flat.json.gz")))["endContent"].encode())
        else:
            want.append(OracleOpLog.load_from(d).checkout_tip_bytes())
    for n in G.JSON_TRACES:
        t = G.trace(n)
        docs.append(dt_amd.apply_edits_push_merge(t["txns"]).encode())
        want.append(t["endContent"].encode())
    # skew: the small traces many times, the big ones twice (configs[4] replicates the set)
    reps = [4, 2, 2, 2, 2, 3, 4, 6]
    batch_docs, batch_want = [], []
    for d, w, r in zip(docs, want, reps):
        batch_docs += [d] * r
        batch_want += [w] * r
    order = sorted(range(len(batch_docs)), key=lambda i: (i * 7919) % len(batch_docs))   # interleaved
    return [batch_docs[i] for i in order], [batch_want[i] for i in order]


def test_mixed_skewed_batch_device_staged(mixed):
    docs, want = mixed
    b = dt_amd.Batch(docs=docs, staging="device")
    b.run()
    b.sync()
    res = b.results()
    lvs = sorted(r["n_lv"] for r in res)
    assert lvs[-1] / lvs[0] > 30                      # skewed
    for i, (r, w) in enumerate(zip(res, want)):
        assert r["status"] == 0, (i, r)
        assert (r["text_len"], r["text_hash"]) == (len(w), dt_amd.text_hash(w)), i
        assert b.text(i) == w, i
    # timed pass over the same resident batch: prep + plan + replay, results unchanged
    ms = b.run_timed()
    assert ms > 0
    assert [(r["status"], r["text_len"], r["text_hash"]) for r in b.results()] == \
           [(0, len(w), dt_amd.text_hash(w)) for w in want]


def test_run_timed_on_host_and_device_staged_batches():
    d = G.dt_bytes("friendsforever")
    for staging in ("host", "device"):
        b = dt_amd.Batch(docs=[d, d, d], staging=staging)
        ms = b.run_timed()
        plan, replay, prep = b.last_times()
        assert ms > 0 and plan > 0 and replay > 0
        assert (prep > 0) == (staging == "device")   # walker inputs are a kernel only when device-staged
        assert all(r["status"] == 0 for r in b.results())


def test_mixed_skewed_batch_forced_segments(mixed, monkeypatch):
    """The same skewed batch with cut replay forced onto every tracker document of 200+ op runs
    (node_nodecc and friendsforever where their histories allow; with DTGPU_FF=0 the linear
    JSON traces too, cut anywhere): segment documents in every LDS tier, the split pass's big
    tier among them, both staging paths; every text still equals its golden / oracle text."""
    monkeypatch.setenv("DTGPU_SEG_OPS", "100")
    docs, want = mixed
    for staging, ff in (("device", "1"), ("host", "1"), ("device", "0")):
        monkeypatch.setenv("DTGPU_FF", ff)
        b = dt_amd.Batch(docs=docs, staging=staging)
        b.run_timed()
        res = b.results()
        for i, (r, w) in enumerate(zip(res, want)):
            assert r["status"] == 0, (staging, i, r)
            assert b.text(i) == w, (staging, i)
        segs = [b.segments(i) for i in range(len(docs))]
        fast = b.fast_forwarded()
        assert (sum(fast) > 0) == (ff == "1")
        tracked = [i for i in range(len(docs)) if not fast[i]]
        assert sum(1 for i in tracked if len(segs[i]) >= 2) >= len(tracked) // 2, staging
        assert all(segs[i] == [] for i in range(len(docs)) if fast[i])
        assert all(x["status"] == 0 for s in segs for x in s)


@pytest.mark.parametrize("critical", ["1", "0"])
def test_configs4_batch_critical_documents(mixed, monkeypatch, critical):
    """configs[4] as bench.py runs it (all 8 traces x 50, round-robin): git-makefile's uncut
    documents are the batch's critical replays (dtgpu_api.cpp mark_critical: first in their
    tier, top wave priority, their tier in the split pipeline with its overlapped walk); with
    DTGPU_CRITICAL=0 none are.  Every text either way equals the golden / oracle text."""
    docs, want = mixed
    uniq = {}
    for d, w in zip(docs, want):
        uniq[d] = w
    names = list(uniq)
    assert len(names) == 8
    monkeypatch.setenv("DTGPU_CRITICAL", critical)
    batch = [names[i % 8] for i in range(400)]
    b = dt_amd.Batch(docs=batch, staging="device")
    b.run()
    b.sync()
    res = b.results()
    for i, r in enumerate(res):
        w = uniq[batch[i]]
        assert r["status"] == 0, (i, r)
        assert (r["text_len"], r["text_hash"]) == (len(w), dt_amd.text_hash(w)), i
    b.run_timed()
    res2 = b.results()
    assert [(r["text_len"], r["text_hash"]) for r in res2] == [(r["text_len"], r["text_hash"]) for r in res]
