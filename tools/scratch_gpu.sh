#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 200 --timeout-method thread > $O/mixtests.log 2>&1
rc=$?; tail -8 $O/mixtests.log; [ $rc -eq 0 ] || exit 1
