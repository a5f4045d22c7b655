"""Device-staged batches (dtgpu_batch_create_device): `.dt` bytes -> GPU decode -> GPU planner
inputs (dt_prep.hip) -> GPU walk plan -> GPU replay.  Same texts as the host-staged path and
the golden / oracle outputs; the device plan equals the host plan command for command."""
import hashlib

import numpy as np
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


def _texts(b):
    b.run()
    b.sync()
    res = b.results()
    return res, [b.text(i) if r["status"] == 0 else None for i, r in enumerate(res)]


def test_friendsforever_device_staged():
    want = G.trace("friendsforever_flat")["endContent"].encode()
    b = dt_amd.Batch(docs=[G.dt_bytes("friendsforever")] * 64, staging="device")
    res, texts = _texts(b)
    assert all(r["status"] == 0 for r in res)
    assert all(t == want for t in texts)
    assert b.host_planned() == [0] * 64


@pytest.mark.parametrize("name", ["git-makefile", "node_nodecc"])
def test_large_docs_device_staged(name):
    data = G.dt_bytes(name)
    b = dt_amd.Batch(docs=[data], staging="device")
    res, texts = _texts(b)
    if res[0]["status"] == dt_amd.DECODE_DEFER:
        pytest.skip("history wider than the device prep limit")
    assert res[0]["status"] == 0
    want = OracleOpLog.load_from(data).checkout_tip_bytes()
    assert hashlib.sha256(texts[0]).hexdigest() == hashlib.sha256(want).hexdigest()


def test_device_plan_equals_host_plan():
    docs = [G.dt_bytes(n) for n in G.DT_FILES]
    dev = dt_amd.Batch(docs=docs, staging="device")
    host = dt_amd.Batch(docs=docs)
    dev.run(); dev.sync(); host.run(); host.sync()
    for i in range(len(docs)):
        if dev.results()[i]["status"] != 0:
            continue
        (dc, dt), (hc, ht) = dev.plan(i), host.plan(i)
        assert np.array_equal(dc, hc), G.DT_FILES[i]
        assert np.array_equal(dt, ht), G.DT_FILES[i]


def test_mixed_errors_and_e2e_rerun():
    good = G.dt_bytes("friendsforever")
    bad = bytearray(good)
    bad[100] ^= 0xFF
    docs = [good, bytes(bad), G.COMPAT_SIMPLE_LZ4, good, b"nope", G.COMPAT_EMPTY_1]
    b = dt_amd.Batch(docs=docs, staging="device")
    h = dt_amd.Batch(docs=docs)
    r1, t1 = _texts(b)
    r2, t2 = _texts(h)
    assert [r["status"] for r in r1] == [r["status"] for r in r2]
    assert t1 == t2
    ms = b.run_e2e_timed()
    assert len(ms) == 4 and all(m > 0 for m in ms)
    r3, t3 = [b.results(), [b.text(i) if r["status"] == 0 else None for i, r in enumerate(b.results())]]
    assert t3 == t1

