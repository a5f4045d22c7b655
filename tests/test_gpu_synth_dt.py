"""Synthetic concurrent documents written as `.dt` (tests/dt_encode.py) through the device
decoder (fast path: ASCII text in known runs; exact path: Unicode text, deleted content,
unknown content) and the device-staged checkout, against the host decoder and the oracle."""
import numpy as np
import pytest

from dt_encode import encode_dt, graph_docs
from oracle.oracle import OpLog as OracleOpLog
from test_dt_encode import WHAT, _unicode

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _docs():
    out = []
    for doc in range(12):
        na, ops = dt_amd.synth_ops(doc, 2000)
        names = [f"a{i}" for i in range(na)]
        kind = doc % 4
        if kind == 1:
            ops = _unicode(ops)
        out.append(encode_dt(names, ops, ins_runs_per_op=(kind == 2), del_content_unknown=(kind == 3)))
    na, ops = dt_amd.synth_ops(99, 1000)
    out.append(encode_dt([f"a{i}" for i in range(na)], ops, unknown_every=7))   # checkout: ErrCheckout
    return out


def test_device_decode_matches_host_on_synthetic_dt():
    docs = _docs()
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        assert dec.status(i)["status"] == 0, i
        host = dt_amd.ListOpLog.load_from(d)
        for w in WHAT:
            a, b = dec.export(i, w), host.export(w)
            assert (a == b) if w == "agent_names" else np.array_equal(a, b), (i, w)


def test_device_staged_checkout_matches_oracle_on_synthetic_dt():
    docs = _docs()
    b = dt_amd.Batch(docs=docs, staging="device")
    b.run()
    b.sync()
    res = b.results()
    for i, d in enumerate(docs):
        if i == len(docs) - 1:   # unknown insert content: the reference cannot check it out
            assert res[i]["status"] != 0
            continue
        assert res[i]["status"] == 0, (i, res[i])
        assert b.text(i) == OracleOpLog.load_from(d).checkout_tip_bytes(), i


def test_device_decode_matches_host_on_graph_shapes():
    docs = graph_docs()
    dec = dt_amd.DecodeBatch(docs)
    dec.run()
    for i, d in enumerate(docs):
        st = dec.status(i)["status"]
        if i == 8:   # the frontier passes 64 elements
            assert st == dt_amd.DECODE_DEFER, i
            continue
        assert st == 0, (i, st)
        host = dt_amd.ListOpLog.load_from(d)
        for w in WHAT:
            a, b = dec.export(i, w), host.export(w)
            assert (a == b) if w == "agent_names" else np.array_equal(a, b), (i, w)
