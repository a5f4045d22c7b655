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


COST_GAMMA = 2.05   # per LV^2 / 1e6: a long document holds a big LDS tier (few per CU) and a long
                    # uncuttable stretch, so its batch cost grows faster than its LVs
COST_BETA = 0.35    # per retreated / advanced LV of the walk plan: lane-parallel toggle passes


def doc_cost(data: bytes) -> float:
    """SURVEY.md 8(e) cost estimate of one document's checkout in a batch, from its host decode
    and host walk plan (native, no GPU): c = LVs + gamma * LVs^2 / 1e6 + beta * walk, walk = LVs
    retreated + advanced by the SpanningTreeWalker plan.  gamma = 2.05 and beta = 0.35 fit the
    per-document batch cost of the eight benchmark traces at round 5 (1,024 device-staged copies
    each, pass ms / 1,024; friendsforever from its 10k pass: profiles/r5_cost/cost_1024.jsonl) to
    within 0.66-1.39x (log least squares); round 2's alpha * runs * log2(runs) term fitted to zero
    and its model was off by up to 4.8x now that cut replay spreads long linear documents over
    waves.  A document that does not decode costs its size."""
    import dt_amd
    try:
        o = dt_amd.ListOpLog.load_from(data)
    except dt_amd.ParseError:   # only an undecodable document; any other error is a bug and raises
        return float(len(data))
    ps = o.plan_stats()
    n = float(len(o))
    return n + COST_GAMMA * n * n / 1e6 + COST_BETA * (ps["retreat"] + ps["advance"])


def gather_results(records, n_total, dist, device=None):
    """All-gather per-document records [(global_index, status, text_len, text_hash), ...] from
    every rank; returns the full table (list of tuples indexed by global document index).
    One all-gather of the counts and one of the padded (n, 4) int64 records (RCCL over xGMI on
    MI355X); the table is scattered with one tensor index per rank, no per-row Python loop."""
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
    rows = torch.cat([b[:int(c.item())] for b, c in zip(bufs, counts)]).cpu()
    rows = rows[rows[:, 0] >= 0]
    full = torch.full((n_total, 4), -1, dtype=torch.int64)
    full[rows[:, 0]] = rows
    have = full[:, 0] >= 0
    out = full.tolist()
    return [tuple(r) if h else None for r, h in zip(out, have.tolist())]


def max_over_ranks(value: float, dist, device=None) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def plan_moves(assign, costs, busy_ms, max_moves=None, tol=0.02):
    """Measured-cost rebalancing of a skewed batch: every rank reports the busy
    time of the same pass; a document's measured cost is its cost estimate times its rank's
    measured ms per estimate unit.  Documents then move, one at a time, from the busiest to the
    idlest rank -- each time the largest one that still narrows the gap -- until the spread is
    within `tol` of the mean or no move helps.  Deterministic: every rank computes the same moves
    from the all-gathered busy times.  Returns (new assignment, [(doc, src, dst), ...])."""
    world = len(assign)
    rate = [busy_ms[r] / max(1e-9, sum(costs[i] for i in assign[r])) for r in range(world)]
    est = {}
    for r in range(world):
        for i in assign[r]:
            est[i] = costs[i] * rate[r]
    load = [float(busy_ms[r]) for r in range(world)]
    parts = [sorted(a, key=lambda i: (est[i], i)) for a in assign]   # ascending measured cost
    moves = []
    limit = max_moves if max_moves is not None else sum(len(a) for a in assign)
    mean = sum(load) / max(1, world)
    while len(moves) < limit:
        src = max(range(world), key=lambda r: (load[r], -r))
        dst = min(range(world), key=lambda r: (load[r], r))
        gap = load[src] - load[dst]
        if gap <= tol * mean or not parts[src]:
            break
        # the documents either side of half the gap; take the one leaving the lower maximum of
        # the pair, if that is below the busiest rank's load
        lo, hi = 0, len(parts[src])
        while lo < hi:
            mid = (lo + hi) // 2
            if est[parts[src][mid]] <= gap / 2:
                lo = mid + 1
            else:
                hi = mid

        def at_dst(i):   # at the destination the document runs at the destination's rate
            return costs[i] * rate[dst] if rate[dst] > 0 else est[i]
        best = None
        for k in (lo - 1, lo):
            if 0 <= k < len(parts[src]):
                i = parts[src][k]
                peak = max(load[src] - est[i], load[dst] + at_dst(i))
                if peak < load[src] - 1e-12 and (best is None or peak < best[0]):
                    best = (peak, k)
        if best is None:
            break
        i = parts[src].pop(best[1])
        c_dst = at_dst(i)
        load[src] -= est[i]
        load[dst] += c_dst
        est[i] = c_dst
        k = 0
        while k < len(parts[dst]) and (est[parts[dst][k]], parts[dst][k]) < (c_dst, i):
            k += 1
        parts[dst].insert(k, i)
        moves.append((i, src, dst))
    return [sorted(p) for p in parts], moves


def exchange_documents(moves, rank, local, dist):
    """Carry out `moves` point to point: the source rank sends each moved document's encoded
    `.dt` bytes (length, then bytes), the destination receives them; `local` maps document index
    -> bytes on this rank and is updated in place.  Every rank walks the same move list, so the
    send/recv pairs match (RCCL over xGMI on MI355X, gloo on CPU)."""
    import torch
    dev = None
    if dist.get_backend() == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    for i, src, dst in moves:
        if rank == src:
            data = local.pop(i)
            n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
            dist.send(n, dst)
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            dist.send(buf.to(dev) if dev is not None else buf, dst)
        elif rank == dst:
            n = torch.zeros(1, dtype=torch.int64, device=dev)
            dist.recv(n, src)
            buf = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
            dist.recv(buf, src)
            local[i] = bytes(buf.cpu().numpy().tobytes())
    return local


def all_gather_floats(value, dist, device=None):
    """Every rank's float (e.g. its busy time), in rank order."""
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]
