"""bench.py's N>1 path, end to end: two ranks launched by torch.distributed.run (the driver's own
command shape), each its own process, both on the box's one GPU (DTGPU_BENCH_SHARED_GPU=1: the
collectives go over gloo instead of RCCL, everything else -- LPT sharding, the barrier +
max-over-ranks timing, the all-gather of per-document (status, len, hash) records checked
against the goldens, the whole-job all-reduce of merged ops, measured rebalancing with .dt bytes
sent point to point -- is the code the 8-GPU run executes)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FF_LV = 26078        # friendsforever.dt: ListOpLog::len()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra, nproc=2, shared=True):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if shared:
        env["DTGPU_BENCH_SHARED_GPU"] = "1"
    else:
        env.pop("DTGPU_BENCH_SHARED_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-encode", "--gen-threads", "4"] + extra
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]   # rank 0 alone prints the line
    return json.loads(lines[0])


@pytest.mark.timeout(480)
def test_bench_two_ranks_friendsforever():
    out = _run(["--docs", "200"])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["scaling"] == "weak"
    assert out["total_merged_ops"] == 2 * 200 * FF_LV
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["docs_per_gpu"] == 200
    assert out["e2e"]["total_ms"] > 0


@pytest.mark.timeout(480)
def test_bench_two_ranks_mixed_rebalance():
    out = _run(["--workload", "mixed", "--docs", "24", "--rebalance"])
    assert out["n_gpus"] == 2
    assert out["config"]["distinct_docs"] == 8
    rb = out["rebalance"]
    assert len(rb["busy_ms_before"]) == 2 and len(rb["busy_ms_after"]) == 2
    assert out["total_merged_ops"] > 0 and out["value"] > 0


@pytest.mark.timeout(480)
@pytest.mark.parametrize("extra", [["--docs", "200"], ["--workload", "mixed", "--docs", "24", "--rebalance"]])
def test_bench_rccl_one_rank(extra):
    """The RCCL code path, run once on the box: torch.distributed.run starts one rank (a fresh
    process, before any GPU call), bench.py joins an `nccl` (RCCL) process group on cuda:0 and runs
    max_over_ranks, gather_results (the per-document table, checked against the goldens / oracle
    inside bench.py) and -- with --rebalance -- all_gather_floats on device tensors."""
    out = _run(extra, nproc=1, shared=False)
    c = out["collectives"]
    assert c["backend"] == "nccl" and c["device"] == "cuda:0" and c["world"] == 1
    assert c["gathered_docs"] == c["gathered_ok"] == int(extra[extra.index("--docs") + 1])
    if "--rebalance" in extra:
        assert len(out["rebalance"]["busy_ms_before"]) == 1 and out["rebalance"]["moves"] == 0
        assert out["total_merged_ops"] > 0
    else:
        assert out["total_merged_ops"] == 200 * FF_LV
