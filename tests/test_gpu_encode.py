""".dt encoding on the GPU side of the engine.

`encode_from(v, ENCODE_FULL)` (src/list/encoding/encode_oplog.rs:404-747, options :122-130) stores
the checkout at `v` in the StartBranch (:606-618); libdtgpu runs that checkout on the device.  The
StartBranch content is the first field appended to the LZ4 buffer, so the decompressed buffer
starts with the device checkout, which must equal the oracle's checkout at `v`.
"""
import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog
from test_encoder import _lz4_chunk, _oracle_lz4_decompress

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if dt_amd.device_count() < 1:
        pytest.fail("no HIP device visible: the engine has no CPU fallback")


@pytest.mark.parametrize("name,frac", [("friendsforever", 0.46), ("git-makefile", 0.3)])
def test_encode_from_full_stores_the_start_branch_checkout(name, frac):
    data = G.dt_bytes(name)
    o = dt_amd.ListOpLog.load_from(data)
    v = [int(len(o) * frac)]
    full = o.encode_from(v)                      # ENCODE_FULL
    patch = o.encode_from(v, dt_amd.ENCODE_PATCH)
    assert len(full) > len(patch)
    expect = OracleOpLog.load_from(data).checkout_bytes(v)
    ul, block = _lz4_chunk(full)
    raw = _oracle_lz4_decompress(block, ul)
    assert raw[:len(expect)] == expect
    assert raw[:len(expect)] == o.checkout_bytes(v)
    # the patch applies on top of the history at v either way
    for p in (full, patch):
        d = dt_amd.ListOpLog.load_from(o.history(v).encode())
        assert d.decode_and_add(p) == o.local_frontier()
        assert d.checkout_tip_bytes() == o.checkout_tip_bytes()
