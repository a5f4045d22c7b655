#!/bin/bash
# Scratch GPU step (edited per experiment; inside gpurun): bash tools/scratch_gpu.sh
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
cat > /tmp/one.py <<'PY'
import sys, os
sys.path.insert(0, "diamond-types_amd"); sys.path.insert(0, "tests")
import dt_amd, golden_data as G
name = sys.argv[1]
data = G.dt_bytes(name) if name in G.DT_FILES else dt_amd.apply_edits_push_merge(G.trace(name)["txns"]).encode()
b = dt_amd.Batch(docs=[data], staging="device"); b.run(); b.sync()
print(name, "ms", min(b.run_timed() for _ in range(3)), "segments", len(b.segments(0)))
PY
for t in automerge-paper rustcode; do
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -f csv -- python -u /tmp/one.py $t > $O/tr.log 2>&1 || exit 1
grep " ms " $O/tr.log
python tools/timeline.py $O/tr/run_kernel_trace.csv
rm -rf $O/tr
done
