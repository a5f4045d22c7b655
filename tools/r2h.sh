#!/bin/bash
OUT=${1:-gpurun_out/r2h}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
for v in lib lib_w5; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_$v.log" 2>&1; echo "$v: $(cat $OUT/kbench_$v.log)"
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kprof.py --plan friendsforever friendsforeverx10000 git-makefile > "$OUT/plan_$v.log" 2>&1; cat "$OUT/plan_$v.log"
done
timeout -k 10 120 python -u tools/dbench.py friendsforever 10000 3 > "$OUT/dbench.log" 2>&1; cat "$OUT/dbench.log"
