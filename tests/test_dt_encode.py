"""The test-side `.dt` writer (tests/dt_encode.py) round-trips synthetic documents: the host
decoder and the oracle decoder read back exactly the oplog the builder API constructs."""
import numpy as np
import pytest

import dt_amd
from dt_encode import encode_dt
from oracle.oracle import OpLog as OracleOpLog

WHAT = ["ops", "agent_runs", "entries", "parent_offsets", "parents", "content", "char_offsets", "version",
        "agent_names"]


def _unicode(ops):
    g = lambda t: "".join(chr(0x3B1 + ord(c) - 97) if i % 2 else chr(0x4E00 + ord(c)) for i, c in enumerate(t))
    return [(a, k, p, n, g(t) if k == 0 else t, par) for a, k, p, n, t, par in ops]


def _builder(n_agents, ops):
    o = dt_amd.ListOpLog()
    ids = [o.get_or_create_agent_id(f"a{i}") for i in range(n_agents)]
    for a, k, p, n, t, par in ops:
        if k == 0:
            o.add_insert_at(ids[a], par, p, t)
        else:
            o.add_delete_at(ids[a], par, p, p + n)
    return o


@pytest.mark.parametrize("doc", [0, 1, 7])
@pytest.mark.parametrize("uni", [False, True])
def test_roundtrip_host_decoder(doc, uni):
    na, ops = dt_amd.synth_ops(doc, 1500)
    if uni:
        ops = _unicode(ops)
    data = encode_dt([f"a{i}" for i in range(na)], ops, ins_runs_per_op=(doc == 1))
    dec = dt_amd.ListOpLog.load_from(data)
    ref = _builder(na, ops)
    for w in WHAT:
        a, b = dec.export(w), ref.export(w)
        assert (a == b) if w == "agent_names" else np.array_equal(a, b), w
    assert len(OracleOpLog.load_from(data)) == len(ref)   # the oracle's decoder accepts it too


def test_unknown_and_deleted_content_decode():
    na, ops = dt_amd.synth_ops(3, 800)
    data = encode_dt([f"a{i}" for i in range(na)], ops, del_content_unknown=True)
    assert len(dt_amd.ListOpLog.load_from(data)) == sum(o[3] for o in ops)
    data2 = encode_dt([f"a{i}" for i in range(na)], ops, unknown_every=5)
    o2 = dt_amd.ListOpLog.load_from(data2)
    with pytest.raises(dt_amd.ParseError):
        o2.checkout_tip()


def test_graph_shape_docs_host_matches_oracle():
    """The OpParents stress documents (dt_encode.graph_docs): the host decoder and the oracle
    read the same history; parent lists come back sorted whatever order they were written in."""
    from dt_encode import graph_docs
    for d in graph_docs():
        host = dt_amd.ListOpLog.load_from(d)
        orc = OracleOpLog.load_from(d)
        assert len(host) == len(orc)
        poff, par = host.export("parent_offsets"), host.export("parents")
        for a, b in zip(poff[:-1], poff[1:]):
            assert list(par[a:b]) == sorted(par[a:b])
