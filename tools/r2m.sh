#!/bin/bash
# planner loads without exec branches: lib (all, incl. row loads) / lib_pa (row loads kept
# guarded) / lib_old (HEAD)
OUT=${1:-gpurun_out/r2m}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
for v in lib lib_pa lib_old lib lib_pa lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_$v.log" 2>&1 || exit 1; echo "$v: $(cut -c1-200 $OUT/kbench_$v.log)"
done
for v in lib lib_pa lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py git-makefile 1000 3 > "$OUT/kbench_gm_$v.log" 2>&1 || exit 1; echo "gm $v: $(cut -c1-200 $OUT/kbench_gm_$v.log)"
done
