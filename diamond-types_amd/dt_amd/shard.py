"""Multi-GPU sharding of independent documents.

Documents never split across GPUs: each rank checks out its own shard.  The only collective
exchanges are (a) the all-gather of per-document (index, status, length, hash) records and
(b) the max-reduce of the timed region -- over RCCL (`nccl` backend) on MI355X, over `gloo` in
the CPU tests.  Shards are assigned by longest-processing-time (LPT) on a per-document cost
estimate so skewed batches (configs[4]) stay balanced.
"""
import heapq


def lpt_assign(costs, world):
    """Greedy LPT: documents by descending cost, each to the currently lightest rank.
    Returns a list of index lists, one per rank (indices ascending within a rank)."""
    loads = [(0, r) for r in range(world)]
    heapq.heapify(loads)
    out = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        load, r = heapq.heappop(loads)
        out[r].append(i)
        heapq.heappush(loads, (load + costs[i], r))
    return [sorted(x) for x in out]


def doc_cost(data: bytes) -> int:
    """Cost proxy before decoding: encoded size (LVs and op runs scale with it)."""
    return len(data)


def gather_results(records, n_total, dist, device=None):
    """All-gather per-document records [(global_index, status, text_len, text_hash), ...] from
    every rank; returns the full table (list of tuples indexed by global document index)."""
    import torch
    world = dist.get_world_size()
    local = torch.tensor([[i, s, l, h & 0x7FFFFFFFFFFFFFFF] for i, s, l, h in records] or [[-1, 0, 0, 0]],
                         dtype=torch.int64, device=device)
    n_local = torch.tensor([len(records)], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(counts, n_local)
    width = max(1, max(int(c.item()) for c in counts))
    pad = torch.full((width, 4), -1, dtype=torch.int64, device=device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad)
    table = [None] * n_total
    for b, c in zip(bufs, counts):
        for row in b[:int(c.item())].tolist():
            if row[0] >= 0:
                table[row[0]] = tuple(row)
    return table


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
