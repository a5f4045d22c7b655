"""Multi-process (world_size 2, gloo, CPU) coverage of the document sharding and the
length/hash gather that the multi-GPU bench performs over RCCL."""
import os
import socket

import pytest

from dt_amd.shard import lpt_assign


def test_lpt_balances_and_covers():
    costs = [100, 1, 1, 1, 50, 50, 7, 3, 3, 90]
    parts = lpt_assign(costs, 3)
    assert sorted(i for p in parts for i in p) == list(range(len(costs)))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)
    assert lpt_assign([5, 5], 4)[2:] == [[], []]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from dt_amd.shard import gather_results, lpt_assign, max_over_ranks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    costs = [(7 * i) % 11 + 1 for i in range(23)]
    mine = lpt_assign(costs, world)[rank]
    # stand-in for the device checkout of this rank's shard: (index, status, len, hash)
    recs = [(i, 0, 1000 + i, (i * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) for i in mine]
    table = gather_results(recs, len(costs), dist)
    t = max_over_ranks(0.5 + rank, dist)
    q.put((rank, table, t))
    dist.destroy_process_group()


def test_gather_over_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, table, t in out:
        assert t == 1.5
        assert [row[0] for row in table] == list(range(23))
        assert all(row[2] == 1000 + row[0] for row in table)
        assert all(row[3] == ((row[0] * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF) & 0x7FFFFFFFFFFFFFFF for row in table)


def test_plan_moves_evens_measured_load():
    from dt_amd.shard import plan_moves
    costs = [10] * 40
    assign = lpt_assign(costs, 4)
    new, moves = plan_moves(assign, costs, [100.0, 100.0, 100.0, 200.0])   # rank 3 runs at half speed
    assert sorted(i for p in new for i in p) == list(range(40))
    assert all(src == 3 for _i, src, _dst in moves) and len(moves) == 4
    rate = [10 / 100, 10 / 100, 10 / 100, 20 / 100]
    loads = [sum(costs[i] * rate[k] for i in p) for k, p in enumerate(new)]
    assert max(loads) < 200 * 0.65
    # balanced input: nothing moves
    assert plan_moves(assign, costs, [100.0] * 4)[1] == []


def _rebalance_worker(rank, world, port, q):
    import torch.distributed as dist
    from dt_amd.shard import all_gather_floats, exchange_documents, lpt_assign, plan_moves
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs = [bytes([i % 251]) * (100 + 37 * i) for i in range(30)]   # stand-ins for .dt files
    costs = [len(d) for d in docs]
    assign = lpt_assign(costs, world)
    local = {i: docs[i] for i in assign[rank]}
    # rank 1 measured three times slower per byte than rank 0
    busy = all_gather_floats(sum(costs[i] for i in assign[rank]) * (3.0 if rank == 1 else 1.0), dist)
    new, moves = plan_moves(assign, costs, busy)
    local = exchange_documents(moves, rank, local, dist)
    q.put((rank, sorted(local), all(local[i] == docs[i] for i in local), new[rank], len(moves)))
    dist.destroy_process_group()


def test_rebalance_exchange_over_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rebalance_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, held0, ok0, new0, m0), (_, held1, ok1, new1, m1) = out
    assert ok0 and ok1 and m0 == m1 > 0
    assert held0 == new0 and held1 == new1
    assert sorted(held0 + held1) == list(range(30))
