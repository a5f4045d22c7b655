#!/bin/bash
OUT=${1:-gpurun_out/r2g}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/kprof.py friendsforever git-makefile node_nodecc > "$OUT/kprof.log" 2>&1; cut -c1-140 "$OUT/kprof.log"
for f in 32 40 44 48 56; do DTGPU_LDS_SB_FILL=$f timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_sb$f.log" 2>&1; echo "fill $f: $(cat $OUT/kbench_sb$f.log)"; done
