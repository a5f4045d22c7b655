#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_mixed.py -x -q --timeout 200 --timeout-method thread > $O/segtests.log 2>&1
rc=$?; tail -3 $O/segtests.log; [ $rc -eq 0 ] || exit 1
for c in 0 1 0 1; do
DTGPU_CRIT_APART=$c timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-encode > $O/mx$c.json 2> $O/mx.err || { tail $O/mx.err; exit 1; }
echo "apart=$c $(grep -o '"ms_per_step": [0-9.]*' $O/mx$c.json)"
done
timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
