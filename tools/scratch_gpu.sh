#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -3 $O/gputests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['bench.py']; import bench
for r in bench.single_doc_table(0, 'device'): print(json.dumps(r))
" > $O/table.log 2>&1 || { tail $O/table.log; exit 1; }
cat $O/table.log
timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
