#!/usr/bin/env python3
"""Batched checkout benchmark (BASELINE.json metric: merged ops/sec for batched checkout).

One step = one device pass of `checkout_tip()` over the whole batch resident in HBM: the
friendsforever.dt workload (BASELINE.json configs[1]) replicated to --docs copies per GPU
(weak scaling: every rank owns its own copies).  The timed pass runs the walker inputs
(dt_prep.hip: parent entries, children CSR, chain decomposition -- what SpanningTreeWalker::new
builds inside checkout_tip, src/listmerge/txn_trace.rs:114-188), the walk planner (dt_plan.hip:
spanning-tree walk + retreat/advance sets) and the replay + materialisation (dt_replay.hip) --
everything the reference's `checkout_tip()` does on a decoded oplog (crates/bench
`complex/merge`).  The `.dt` bytes are decoded on the device too (dt_decode.hip); the reference
benches decode separately (`complex/decode`), so decode is outside the timed pass and the whole
chain -- decode + prep + plan + replay from the encoded bytes -- is reported as `e2e`.

Contract: `python bench.py --gpus N --steps K --warmup W` prints ONE JSON line on rank 0.
For N > 1 it is launched by torch.distributed.run, one process per GPU; per-rank times are
max-reduced over RCCL (`nccl` backend) and per-document (len, hash) records are all-gathered
over RCCL and checked against the golden text, the only collective the path needs.
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "diamond-types_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--docs", type=int, default=10000, help="documents per GPU")
    p.add_argument("--workload", default="friendsforever",
                   help="friendsforever | git-makefile | node_nodecc (benchmark_data copies), synth "
                        "(BASELINE configs[3]: synthetic concurrent documents, dt_synth.cpp, written as .dt) or "
                        "mixed (configs[4]: all 8 benchmark_data traces) or linear (the five linear JSON traces, "
                        "checked out on the fast-forward path, dt_ff.hip)")
    p.add_argument("--distinct", type=int, default=256, help="synth: distinct documents, replicated to --docs")
    p.add_argument("--synth-family", default="merge", choices=["merge", "epoch"],
                   help="synth: SURVEY 8(d)4 pairwise-merge generator (default) or the epoch generator")
    p.add_argument("--rebalance", action="store_true",
                   help="N>1: move documents from busy to idle ranks by measured cost before timing")
    p.add_argument("--gen-threads", type=int, default=16, help="host threads generating / checking distinct documents")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    p.add_argument("--cpu-cores", type=int, default=0,
                   help="host threads of the CPU baseline (0: the host CPUs this process may use, "
                        "capped by the job's CPU share -- cgroup quota / OMP_NUM_THREADS)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-decode", action="store_true", help="skip the end-to-end (.dt bytes -> text) measurement")
    p.add_argument("--no-encode", action="store_true", help="skip the batched encoder (oplogs -> .dt) measurement")
    p.add_argument("--host-staging", action="store_true", help="decode and prepare planner inputs on host threads")
    return p.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Threads for the CPU baseline: the CPUs this process may run on (hardware_concurrency as
    the affinity mask sees it), capped by the job's CPU share -- the cgroup cpu.max quota and
    OMP_NUM_THREADS, which the GPU box sets to its per-GPU share.  Returns (threads, why)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = [f"affinity {n}"]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
            why.append(f"cgroup quota {int(q) / int(per):g}")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        why.append(f"OMP_NUM_THREADS {omp}")
    return max(1, n), ", ".join(why)


def cpu_baseline(pool, budget_s, cores, workload="friendsforever"):
    """The CPU oracle (C restatement of the reference algorithm, one document per thread)
    timed on a bounded sample of the same workload: checkout_tip() on an already-decoded
    oplog, as the reference's `complex/merge` bench times it.  `pool`: the distinct documents.
    A linear history takes the oracle's fast-forward path (dto_checkout_tip_ff, as the
    reference's merge.rs:811-840); a concurrent one replays every LV through a per-item tracker
    where the reference uses RLE spans, so on concurrent histories the real Rust path is likely
    faster than this restatement."""
    from oracle.oracle import OpLog as OracleOpLog
    why = "--cpu-cores"
    if cores <= 0:
        cores, why = host_threads()
    o = OracleOpLog.load_from(pool[0])
    t0 = time.perf_counter()
    o.checkout_tip_ff_bytes()
    one = time.perf_counter() - t0
    per_core = max(1, int(budget_s / max(one, 1e-4) / cores))
    done = [0] * cores
    lvs = [0] * cores
    ff = [False] * cores
    logs = [[OracleOpLog.load_from(pool[(k + j) % len(pool)]) for j in range(min(len(pool), 4))] for k in range(cores)]

    def work(k):
        for i in range(per_core):
            lg = logs[k][i % len(logs[k])]
            ff[k] |= lg.checkout_tip_ff_bytes()[1]
            done[k] += 1
            lvs[k] += len(lg)

    th = [threading.Thread(target=work, args=(k,)) for k in range(cores)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    docs = sum(done)
    return {"value": sum(lvs) / wall, "unit": "merged ops/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "threads_from": why,
            "sample": f"{docs} x {workload} checkout_tip (decoded oplog) on {cores} host threads, {wall:.2f} s: "
                      f"C restatement of the reference algorithm (oracle/dt_oracle.c): "
                      + ("the fast-forward path for the linear histories (dto_checkout_tip_ff, merge.rs:811-840)"
                         + (", the per-item tracker for the others" if len(pool) > 5 else "") if any(ff) else
                         "per-item tracker (no linear history in the sample; the reference fast-forwards only a "
                         "linear prefix, merge.rs:811-840)")}


def cpu_config0():
    """BASELINE configs[0]: automerge-paper.json.gz -> ListOpLog (untimed, the
    apply_edits_push_merge construction of crates/bench/src/utils.rs:25-44) -> checkout_tip on
    one host core, median of 5 after one warmup (criterion-style; bench.sh:5-7 pins one core).
    The history is linear, so the reference's checkout is all fast-forward (merge.rs:811-840):
    the oracle's FF path (dto_checkout_tip_ff) is the baseline; its per-item tracker is timed
    beside it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_data as G
    from oracle.oracle import oplog_from_trace
    t = G.trace("automerge-paper")
    o = oplog_from_trace(t["txns"])
    want = t["endContent"].encode()

    def med(fn):
        fn()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[2], out
    ff_s, (text, ff) = med(o.checkout_tip_ff_bytes)
    assert ff and text == want, "automerge-paper FF checkout differs from endContent"
    tr_s, text2 = med(o.checkout_tip_bytes)
    assert text2 == want, "automerge-paper tracker checkout differs from endContent"
    return {"workload": "automerge-paper.json.gz -> checkout_tip (BASELINE configs[0])", "merged_ops": len(o),
            "ff_ms": ff_s * 1e3, "ff_merged_ops_per_s": len(o) / ff_s,
            "tracker_ms": tr_s * 1e3, "tracker_merged_ops_per_s": len(o) / tr_s,
            "cores": 1, "cpu_model": cpu_model(), "stat": "median of 5 after 1 warmup",
            "text_bytes": len(want), "checked": "endContent"}


def single_doc_latency(data, gpu, staging):
    """One document alone (single-doc latency on one core, median of 5 after a
    warmup): the GPU checkout pass of a one-document batch next to the C oracle's checkout_tip()
    on one host thread.  A document's replay is a sequential chain between the cut points of its
    history; the cut replay (dt_replay.hip "segments") runs the pieces on separate waves."""
    import dt_amd
    from oracle.oracle import OpLog as OracleOpLog
    b = dt_amd.Batch(docs=[data], device=gpu, staging=staging)
    b.run()
    b.sync()
    g = sorted(b.run_timed() for _ in range(5))[2]
    o = OracleOpLog.load_from(data)
    o.checkout_tip_bytes()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        o.checkout_tip_bytes()
        ts.append((time.perf_counter() - t0) * 1000.0)
    return {"gpu_ms": g, "cpu_ms": sorted(ts)[2], "cpu_cores": 1, "doc": "first document of the workload"}


def single_doc_table(gpu, staging):
    """SURVEY.md 8(d) single-document latency for every benchmark_data trace (bench.sh:5-7 pins
    one core): the GPU checkout pass of a one-document batch (median of 5 after a warmup) next
    to the C oracle's checkout_tip on one host thread, fast-forwarding a linear history as the
    reference does (dto_checkout_tip_ff, merge.rs:811-840; the tracker otherwise).  `cut_ms` is
    the host's cut analysis for the document (dtgpu_oplog_cut_ranges: where the history is one
    version, the boundary the reference fast-forwards across), which staging runs before the
    pass when it replays the document as segments; `gpu_with_cut_ms` counts it in.  Every text
    is checked: the .dt files against the oracle, the JSON traces against their endContent."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_data as G
    import dt_amd
    from oracle.oracle import OpLog as OracleOpLog, oplog_from_trace
    rows = []

    def med(fn, k=5):
        fn()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            out = fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[k // 2], out
    for name in list(G.DT_FILES) + list(G.JSON_TRACES):
        if name in G.DT_FILES:
            data = G.dt_bytes(name)
            o = OracleOpLog.load_from(data)
            want = None
        else:
            t = G.trace(name)
            data = dt_amd.apply_edits_push_merge(t["txns"]).encode()
            o = oplog_from_trace(t["txns"])
            want = t["endContent"].encode()
        cpu_ms, (text, ff) = med(o.checkout_tip_ff_bytes)
        if want is None:
            want = text
        assert text == want, f"{name}: oracle checkout differs"
        b = dt_amd.Batch(docs=[data], device=gpu, staging=staging)
        b.run()
        b.sync()
        g = sorted(b.run_timed() for _ in range(5))[2]
        assert b.results()[0]["status"] == 0 and b.text(0) == want, f"{name}: GPU checkout differs"
        h = dt_amd.ListOpLog.load_from(data)
        cut_ms, _ = med(h.cut_ranges)
        segs = len(b.segments(0))
        rows.append({"trace": name, "merged_ops": len(o), "gpu_ms": g, "cut_ms": cut_ms,
                     "gpu_with_cut_ms": g + (cut_ms if segs else 0.0), "segments": segs,
                     "cpu_ms": cpu_ms, "cpu_path": "fast-forward" if ff else "tracker", "cpu_cores": 1})
    return rows


def cold_leg(docs, gpu, staging, expect, runs=1):
    """Cold path: a fresh batch of the same documents, `.dt` bytes in host memory
    -> staging (upload, device decode, prep, planner sizing, cut sizing, arenas) -> the first
    checkout pass -> texts in HBM, wall clock; the process's HIP runtime is already initialised
    (the first batch's `stage_s` includes that).  `runs` fresh batches one after another: the
    median run is reported, with every run's total listed.  One by default: a second and third
    fresh batch of 10,000 documents in the same process sometimes took 1-1.7 s (allocation after
    the previous cold batch's release), which is not the cold path of a fresh batch."""
    legs = sorted((cold_once(docs, gpu, staging, expect) for _ in range(max(1, runs))), key=lambda x: x["cold_ms"])
    out = dict(legs[len(legs) // 2])
    out["cold_ms_runs"] = [round(x["cold_ms"], 2) for x in legs]
    return out


def cold_once(docs, gpu, staging, expect):
    import dt_amd
    t0 = time.perf_counter()
    b = dt_amd.Batch(docs=docs, device=gpu, staging=staging)
    t1 = time.perf_counter()
    ms = b.run_timed()
    b.sync()
    t2 = time.perf_counter()
    res = b.results()
    bad = sum(1 for r, w in zip(res, expect) if r["status"] != 0 or (r["text_len"], r["text_hash"]) != w)
    assert bad == 0, f"cold batch: {bad} documents differ"
    del b
    return {"stage_ms": (t1 - t0) * 1e3, "first_pass_ms": ms, "cold_ms": (t2 - t0) * 1e3,
            "basis": "fresh batch of the workload's documents: bytes in host memory -> texts in HBM, staging included"}


def e2e_leg(batch, docs, steps, expect, total_lv):
    """`.dt` bytes in HBM -> text: device decode (dt_decode.hip) + planner inputs (dt_prep.hip) +
    walk plan + replay, re-run `steps` times on the device-staged batch (HIP events per kernel).
    Roofline basis = SURVEY.md 8d E2E: encoded bytes + text bytes per document.  The decoder's
    arrays are parity-checked against the host decoder on document 0."""
    import dt_amd
    split = [batch.run_e2e_timed() for _ in range(max(1, steps))]
    res = batch.results()
    assert all(r["status"] == 0 and (r["text_len"], r["text_hash"]) == e for r, e in zip(res, expect)), \
        "end-to-end results differ"
    dec = dt_amd.DecodeBatch(docs[:1])
    dec.run()
    host = dt_amd.ListOpLog.load_from(docs[0])
    for w in ("ops", "agent_runs", "entries", "parents", "char_offsets", "content"):
        assert (dec.export(0, w) == host.export(w)).all(), w
    mean = [statistics.mean(x[k] for x in split) for k in range(4)]
    total = sum(mean)
    enc = sum(len(d) for d in docs)
    basis = enc + sum(e[0] for e in expect)
    return {"decode_ms": mean[0], "prep_ms": mean[1], "plan_ms": mean[2], "replay_ms": mean[3], "total_ms": total,
            "merged_ops_per_s": total_lv / (total / 1000.0), "docs_per_s": len(docs) / (total / 1000.0),
            "encoded_bytes": enc, "roofline_bytes": basis,
            "achieved_GBps": basis / (total / 1000.0) / 1e9, "frac_hbm": basis / (total / 1000.0) / 1e9 / HBM_PEAK_GBS,
            "basis": "SURVEY.md 8d E2E: |.dt bytes| + |text out| per document; kernel time of decode + prep + plan + replay"}


def encode_leg(batch, docs, steps, cpu_budget_s, cores):
    """SURVEY.md 8(f)2, the `.dt` encoder: ListOpLog::encode(ENCODE_FULL) from ROOT for every
    document of the resident batch on the GPU (dt_encoder.hip: records kernel + LZ4/write
    kernel, HIP events), bytes checked against the host encoder on the first and last document.
    Roofline basis: decoded SoA bytes read + `.dt` bytes written.  CPU baseline: the host encoder
    (C++ restatement of encode_oplog.rs + lz4_flex's compressor) on a bounded sample, one
    document per host thread."""
    import dt_amd
    ms = [batch.encode() for _ in range(max(1, steps))]
    n_docs = len(docs)
    staged = [i for i in (0, n_docs - 1) if batch.encoded_status(i) == 0]   # deferred documents have no bytes
    for i in staged:
        assert batch.encoded(i) == dt_amd.ListOpLog.load_from(docs[i]).encode(), "device encoder bytes differ from the host encoder's"

    out_b, in_b = batch.encoded_bytes(0), batch.encoded_bytes(1)
    t = statistics.mean(ms)
    logs = [dt_amd.ListOpLog.load_from(d) for d in docs[:8]]
    t0 = time.perf_counter()
    logs[0].encode()
    one = time.perf_counter() - t0
    if cores <= 0:
        cores, _ = host_threads()
    per = max(1, int(cpu_budget_s / max(one, 1e-4) / cores))
    done = [0] * cores

    def work(k):
        for i in range(per):
            logs[(k + i) % len(logs)].encode()
            done[k] += 1
    th = [threading.Thread(target=work, args=(k,)) for k in range(cores)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    return {"kernel_ms": t, "docs_per_s": n_docs / (t / 1000.0), "encoded_bytes": out_b, "soa_bytes_read": in_b,
            "achieved_GBps": (out_b + in_b) / (t / 1000.0) / 1e9,
            "frac_hbm": (out_b + in_b) / (t / 1000.0) / 1e9 / HBM_PEAK_GBS,
            "checked": f"bytes of documents {staged} equal dtgpu_oplog_encode (host)",
            "cpu_baseline": {"docs_per_s": sum(done) / wall, "cores": cores, "kind": "port",
                             "sample": f"{sum(done)} host encodes (dtgpu_oplog_encode, ENCODE_FULL) on {cores} threads, "
                                       f"{wall:.2f} s"}}


def workload_pool(args):
    """The distinct documents of the workload (raw `.dt` bytes) and the `data` description."""
    if args.workload == "synth":
        import dt_amd
        from concurrent.futures import ThreadPoolExecutor

        def gen(d):   # generator and encoder are native (ctypes releases the GIL)
            if args.synth_family == "epoch":
                return dt_amd.synth_oplog(d, 5000).encode()
            return dt_amd.synth_merge_oplog(d, 5000).encode()
        pool = []
        with ThreadPoolExecutor(max(1, args.gen_threads)) as ex:
            for c in range(0, args.distinct, 4096):   # progress on stderr for long pools
                pool += list(ex.map(gen, range(c, min(args.distinct, c + 4096))))
                if args.distinct > 4096:
                    print(f"[bench] generated {len(pool)}/{args.distinct} distinct documents", file=sys.stderr, flush=True)
        fam = ("epoch merges (dtgpu_synth_oplog)" if args.synth_family == "epoch" else
               "SURVEY 8(d)4: per-step pairwise merges p=0.1 via find_dominators_2 (dtgpu_synth_merge_oplog)")
        return pool, (f"synthetic concurrent documents (dt_synth.cpp: seed 0xD1A00000 + doc, 4-16 agents, "
                      f"~5k ops, {fam}), {args.distinct} distinct encoded as .dt (dtgpu_oplog_encode) "
                      f"and replicated")
    if args.workload == "mixed":   # BASELINE configs[4]: all benchmark_data traces, skewed sizes
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import golden_data as G
        import dt_amd
        pool = [open(os.path.join(ROOT, "tests", "golden", "benchmark_data", n + ".dt"), "rb").read()
                for n in G.DT_FILES]
        for name in G.JSON_TRACES:   # oplog as crates/bench builds it, encoded by the native encoder
            pool.append(dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode())
        return pool, ("all 8 benchmark_data traces (3 .dt files + 5 JSON traces built the way "
                      "crates/bench/src/utils.rs:25-44 builds their oplogs and written as .dt by "
                      "dtgpu_oplog_encode), replicated round-robin")
    if args.workload == "linear":   # the five linear traces: one graph entry each (fast-forward path)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import golden_data as G
        import dt_amd
        pool = [dt_amd.apply_edits_push_merge(G.trace(n)["txns"]).encode() for n in G.JSON_TRACES]
        return pool, ("the 5 linear benchmark_data JSON traces (automerge-paper, rustcode, seph-blog1, "
                      "sveltecomponent, friendsforever_flat) built as crates/bench/src/utils.rs:25-44 builds "
                      "them, written as .dt by dtgpu_oplog_encode, replicated round-robin")
    path = os.path.join(ROOT, "tests", "golden", "benchmark_data", args.workload + ".dt")
    return [open(path, "rb").read()], f"benchmark_data/{args.workload}.dt replicated (byte-identical copies in distinct buffers)"


def expected_texts(args, pool):
    """(len, hash) of the reference's checkout per distinct document: friendsforever's golden
    endContent; otherwise the C oracle (a bounded number of distinct documents)."""
    import dt_amd
    if args.workload == "friendsforever":
        import gzip
        gold = json.load(gzip.open(os.path.join(ROOT, "tests", "golden", "benchmark_data",
                                                "friendsforever_flat.json.gz")))["endContent"].encode()
        return [(len(gold), dt_amd.text_hash(gold))]
    from oracle.oracle import OpLog as OracleOpLog
    from concurrent.futures import ThreadPoolExecutor

    def one(d):
        t = OracleOpLog.load_from(d).checkout_tip_ff_bytes()[0]   # (the tracker unless linear)
        return (len(t), dt_amd.text_hash(t))
    with ThreadPoolExecutor(max(1, args.gen_threads)) as ex:
        return list(ex.map(one, pool))


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # a process group whenever the launcher started us (torch.distributed.run sets
    # TORCHELASTIC_RUN_ID), also at one rank: the RCCL collectives then run on cuda:0
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:
        import torch
        import torch.distributed as dist
        # rehearsal of the N-rank path on a 1-GPU box: every rank on GPU 0, collectives over gloo
        shared = os.environ.get("DTGPU_BENCH_SHARED_GPU") == "1"
        gpu = 0 if shared else local_rank
        torch.cuda.set_device(gpu)
        dist.init_process_group("gloo" if shared else "nccl")

    import dt_amd
    from dt_amd.shard import doc_cost, gather_results, lpt_assign, max_over_ranks
    pool, data_desc = workload_pool(args)
    n_total = args.docs * world
    # weak scaling: the global batch is docs x world documents (document g is pool[g % distinct]);
    # LPT gives every rank its shard
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max(1, args.gen_threads)) as ex:   # per distinct document, native (GIL released)
        pool_cost = list(ex.map(doc_cost, pool))
    mine = lpt_assign([pool_cost[g % len(pool)] for g in range(n_total)], world)[rank]
    docs = [bytes(pool[g % len(pool)]) for g in mine]
    gpu = 0 if (dist is None or os.environ.get("DTGPU_BENCH_SHARED_GPU") == "1") else local_rank
    dev = (None if os.environ.get("DTGPU_BENCH_SHARED_GPU") == "1" else f"cuda:{local_rank}") if dist is not None else None

    t0 = time.perf_counter()
    staging = "host" if args.host_staging else "device"
    batch = dt_amd.Batch(docs=docs, device=gpu, staging=staging)
    host_stage_s = time.perf_counter() - t0

    for _ in range(args.warmup):
        batch.run()
    batch.sync()

    rebalance = None
    if dist is not None and args.rebalance:
        # measured-cost rebalancing: all-gather each rank's busy time for one
        # pass, plan the moves identically on every rank, send the moved documents' .dt bytes
        # point to point and re-stage (all outside the timed region)
        from dt_amd.shard import all_gather_floats, exchange_documents, plan_moves
        costs = [pool_cost[g % len(pool)] for g in range(n_total)]
        assign = lpt_assign(costs, world)
        busy = all_gather_floats(batch.run_timed(), dist, device=dev)
        new_assign, moves = plan_moves(assign, costs, busy, tol=0.10)   # spreads under 10 % are noise
        local = exchange_documents(moves, rank, dict(zip(mine, docs)), dist)
        mine = new_assign[rank]
        docs = [local[g] for g in mine]
        if moves:
            del batch
            batch = dt_amd.Batch(docs=docs, device=gpu, staging=staging)
            for _ in range(max(1, args.warmup)):
                batch.run()
            batch.sync()
        after = all_gather_floats(batch.run_timed(), dist, device=dev)
        rebalance = {"moves": len(moves), "busy_ms_before": busy, "busy_ms_after": after}

    # timed region: K device checkout passes (prep + plan + replay) over the resident batch
    kernel_ms, split = [], []
    batch.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kernel_ms.append(batch.run_timed())
        split.append(batch.last_times())
    batch.sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = max_over_ranks(elapsed, dist, device=dev)
        dist.barrier()

    # correctness gate (outside the timed region, on the last timed pass's output, so that a
    # --warmup 0 profiling run checks real results): every document's text equals the golden
    res = batch.results()
    gold = expected_texts(args, pool)   # golden endContent / oracle checkout per distinct document
    want = [gold[g % len(pool)] for g in mine]
    bad = sum(1 for r, w in zip(res, want) if r["status"] != 0 or (r["text_len"], r["text_hash"]) != w)
    assert bad == 0, f"{bad} documents differ from the golden / oracle text"
    total_lv_mine = sum(r["n_lv"] for r in res)
    total_lv = total_lv_mine
    collectives = None
    if dist is not None:   # RCCL all-gather of per-document (len, hash) records
        table = gather_results([(g, r["status"], r["text_len"], r["text_hash"]) for g, r in zip(mine, res)],
                               n_total, dist, device=dev)
        assert all(row is not None and row[1] == 0 and row[2] == gold[row[0] % len(pool)][0] for row in table), \
            "gather mismatch"
        import torch
        t = torch.tensor([float(total_lv_mine)], dtype=torch.float64, device=dev)
        dist.all_reduce(t)   # whole-job merged ops
        total_lv = int(t.item())
        dist.barrier()
        collectives = {"backend": dist.get_backend(), "device": str(dev) if dev is not None else "cpu",
                       "world": world, "gathered_docs": len(table),
                       "gathered_ok": sum(1 for row in table if row is not None and row[1] == 0)}
    lv_per_doc = total_lv_mine / max(1, len(mine))
    ms_per_step = elapsed * 1000.0 / args.steps
    value = total_lv * args.steps / elapsed
    avg_kernel_ms = statistics.mean(kernel_ms)
    plan_ms = statistics.mean(x[0] for x in split)
    replay_ms = statistics.mean(x[1] for x in split)
    prep_ms = statistics.mean(x[2] for x in split)
    alg_bytes = batch.algorithmic_bytes
    n_ff = sum(batch.fast_forwarded())
    all_ff = n_ff == len(docs)
    # roofline of the dominant kernel (replay_kernel): the pass's algorithmic bytes over the
    # replay launch's own HIP-event time on the batch's stream
    achieved = alg_bytes / (replay_ms / 1000.0) / 1e9
    traffic = pass_traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.workload}_{args.docs}.json")
    if os.path.exists(tpath):   # HBM bytes per launch from rocprofv3 PMC runs of this command
        tj = json.load(open(tpath))
        pass_traffic = tj.get("hbm_bytes_per_pass")
        rk = [v for k, v in tj.get("per_kernel", {}).items() if k.startswith("ff_" if all_ff else "replay_kernel")]
        if rk:   # every replay tier's launch of the pass (tools/traffic.py)
            traffic = sum(2 * v["fetch_kib"] + v["write_kib"] for v in rk) * 1024

    out = {
        "metric": "merged ops/sec (whole node) for batched checkout",
        "value": value,
        "unit": "merged ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32/u8 integer",
        "data": data_desc,
        "config": {"workload": f"{args.workload} x {args.docs} docs per GPU (checkout_tip)",
                   "docs_per_gpu": args.docs, "merged_ops_per_doc": lv_per_doc,
                   "distinct_docs": len(pool),
                   "timed": ("fast-forward checkout (dt_ff.hip: segment replays on piece tables, pairwise "
                             "composition, text) of the whole batch (decoded oplogs resident in HBM)" if all_ff else
                             "device walker inputs (prep) + cut planning + walk planning + replay + materialisation "
                             "of the whole batch (decoded oplogs resident in HBM)"
                             + (f"; {n_ff} linear documents on the fast-forward path (dt_ff.hip)" if n_ff else "")),
                   "parallelism": f"dp{world} (documents sharded, no data-path collective)"},
        "docs_per_sec": n_total * args.steps / elapsed,
        "total_merged_ops": total_lv,
        "stage_s": host_stage_s,
        "staging": staging,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("ff kernels (dt_ff.hip: delta, segment replay, composition levels, text, copy)"
                                if all_ff else "replay_kernel (dominant kernel of the pass)"), "kernel_ms": replay_ms,
                     "pass": {"kernels": ("ff_delta + ff_seg + ff_compose x levels + ff_text + ff_copy" if all_ff else
                                          "prep_kernel x2 + chain_kernel + walk_kernel + cut_kernel + plan_kernel + "
                                          "replay_kernel tiers + combine_kernel"
                                          + (" + the ff kernels" if n_ff else "")), "ms": avg_kernel_ms,
                              "prep_ms": prep_ms, "plan_ms": plan_ms, "replay_ms": replay_ms,
                              "achieved": alg_bytes / (avg_kernel_ms / 1000.0) / 1e9,
                              "frac": alg_bytes / (avg_kernel_ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                              "traffic": pass_traffic},
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "algorithmic_formula": "per doc: 16*op_runs + (8+4*parents)*graph_entries + 12*agent_runs "
                                            "+ inserted_bytes + text_out_bytes (SURVEY.md 8d merge-only)"},
    }
    if rebalance is not None:
        out["rebalance"] = rebalance
    if collectives is not None:
        out["collectives"] = collectives
    if not args.no_decode and staging == "device":   # .dt bytes -> text, all on the GPU
        out["e2e"] = e2e_leg(batch, docs, min(args.steps, 5), want, total_lv_mine)
        if rank == 0:   # (with the timed batch still resident: releasing its arenas first made
            # the fresh batches' allocations take up to 1.6 s on some runs)
            out["cold"] = cold_leg(docs, gpu, staging, want)
    if not args.no_encode and staging == "device" and rank == 0:   # oplogs -> .dt bytes on the GPU
        out["encode"] = encode_leg(batch, docs, min(args.steps, 5), 3.0, args.cpu_cores)
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pool, args.cpu_seconds, args.cpu_cores, args.workload)
        out["single_doc_latency"] = single_doc_latency(pool[0], gpu, staging)
        if staging == "device":
            out["single_doc_table"] = single_doc_table(gpu, staging)
        out["cpu_config0"] = cpu_config0()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
