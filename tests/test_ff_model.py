"""CPU checks of the fast-forward checkout's algorithm (tests/ff_model.py, the sequential model of
dt_ff.hip: segments of 63 op runs on piece lists, pairwise composition, byte offsets) against the
reference's own endContent for the five linear benchmark traces and against the oracle's
fast-forward checkout (oracle/dt_oracle.c dto_checkout_tip_ff, merge.rs:811-840) for random
linear histories.  The kernels themselves are checked on the GPU (tests/test_gpu_ff.py)."""
import pytest

import dt_amd
import ff_model
import golden_data as G
import linear_docs as L
from oracle.oracle import OpLog as OracleOpLog


def model_text(data):
    o = dt_amd.ListOpLog.load_from(data)
    assert len(o.export("entries")) <= 1   # one graph entry: the linear case
    return ff_model.checkout(o.export("ops").tolist(), o.export("char_offsets").tolist(), bytes(o.export("content")))


@pytest.mark.parametrize("name", G.JSON_TRACES)
def test_model_matches_end_content(name):
    t = G.trace(name)
    o = dt_amd.apply_edits_push_merge(t["txns"])
    got = ff_model.checkout(o.export("ops").tolist(), o.export("char_offsets").tolist(), bytes(o.export("content")))
    assert got == t["endContent"].encode()


@pytest.mark.parametrize("seed", range(12))
def test_model_matches_oracle_on_random_linear_histories(seed):
    data, want = L.random_linear(seed, 300 + 150 * seed)
    text, ff = OracleOpLog.load_from(data).checkout_tip_ff_bytes()
    assert ff and text == want
    assert model_text(data) == want


@pytest.mark.parametrize("runs", [1, 2, 62, 63, 64, 126, 127, 128, 189, 4000])
def test_model_segment_boundaries(runs):
    data, want = L.sized_linear(runs, seed=runs)
    assert OracleOpLog.load_from(data).checkout_tip_bytes() == want
    assert model_text(data) == want
