#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mx() { timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-encode > $O/mx.json 2> $O/mx.err || { tail $O/mx.err; return 1; }; grep -o '"ms_per_step": [0-9.]*' $O/mx.json; }
for k in 1 2; do
echo "overlap: $(mx)" || exit 1
echo "no overlap: $(DTGPU_NO_WALK_OVERLAP=1 mx)" || exit 1
done
rm -rf $O/mx
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/mx -o run -f csv -- python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-encode > $O/mx.log 2>&1 || { tail $O/mx.log; exit 1; }
