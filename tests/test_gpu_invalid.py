"""Divergent and invalid inputs through the device checkout: every replay loop is bounded (a
step budget per document) and every bad operation ends its document with a status, never a hang
or a batch abort.  Random op streams with random parents and positions that often fall outside
the document (the reference panics there: merge.rs:384, 489; yjsspan.rs:49-90) must give the
oracle's verdict per document: the same text where it checks out, ErrCheckout where it panics."""
import random

import pytest

import golden_data as G
from oracle.oracle import OpLog as OracleOpLog, OracleError

pytestmark = pytest.mark.gpu

import dt_amd  # noqa: E402

ERR_CHECKOUT = 64


def _random_oplog(seed, n_ops=150):
    rng = random.Random(seed)
    o = dt_amd.ListOpLog()
    agents = [o.get_or_create_agent_id(f"a{i}") for i in range(rng.randint(1, 5))]
    n_lv, approx = 0, 0
    for _ in range(n_ops):
        parents = sorted(set(rng.randrange(n_lv) for _ in range(rng.randint(1, 2)))) if n_lv else []
        pos = rng.randint(0, max(1, int(approx * 1.3) + 2))
        if approx == 0 or rng.random() < 0.6:
            s = "".join(rng.choice("abcxyz") for _ in range(rng.randint(1, 4)))
            r = o.add_insert_at(rng.choice(agents), parents, pos, s)
            approx += len(s)
        else:
            r = o.add_delete_at(rng.choice(agents), parents, pos, pos + rng.randint(1, 3))
            approx = max(0, approx - 1)
        n_lv = len(o)
        assert r >= 0
    return o


def _oracle(data):
    try:
        return OracleOpLog.load_from(data).checkout_tip_bytes()
    except OracleError:
        return None


@pytest.mark.parametrize("staging", ["device", "host"])
def test_random_invalid_oplogs_match_oracle_verdicts(staging):
    docs = []
    for s in range(24):   # random streams (mostly invalid) between valid generated documents
        docs.append(_random_oplog(s).encode())
        docs.append(dt_amd.synth_merge_oplog(500 + s, 800).encode())
    docs.insert(7, G.dt_bytes("friendsforever"))   # a valid, long document among them
    want = [_oracle(d) for d in docs]
    assert 5 < sum(w is None for w in want) < len(docs) - 5, "the mix needs both verdicts"
    b = dt_amd.Batch(docs=docs, staging=staging)
    b.run()
    b.sync()
    res = b.results()
    deferred = [i for i, r in enumerate(res) if r["status"] == dt_amd.DECODE_DEFER]
    assert staging == "device" or not deferred
    for i, (r, w) in enumerate(zip(res, want)):
        if i in deferred:
            continue
        if w is None:
            assert r["status"] == ERR_CHECKOUT, (i, r)
        else:
            assert r["status"] == 0, (i, r)
            assert b.text(i) == w, i
    if deferred:   # the device decoder hands odd documents back: the host-staged retry decides
        h = dt_amd.Batch(docs=[docs[i] for i in deferred], staging="host")
        h.run()
        h.sync()
        for k, i in enumerate(deferred):
            r = h.results()[k]
            if want[i] is None:
                assert r["status"] == ERR_CHECKOUT, (i, r)
            else:
                assert r["status"] == 0 and h.text(k) == want[i], (i, r)


def test_invalid_positions_single_oplog():
    o = dt_amd.ListOpLog()
    a = o.get_or_create_agent_id("x")
    o.add_insert(a, 0, "hello")
    o.add_insert_at(a, [4], 10, "zz")        # past the end of "hello"
    with pytest.raises(dt_amd.ParseError):
        o.checkout_tip_bytes()
    o2 = dt_amd.ListOpLog()
    a = o2.get_or_create_agent_id("x")
    o2.add_insert(a, 0, "abc")
    o2.add_delete_at(a, [2], 2, 9)           # deletes past the end
    with pytest.raises(dt_amd.ParseError):
        o2.checkout_tip_bytes()
