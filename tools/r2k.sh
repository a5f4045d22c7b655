#!/bin/bash
# level-synchronous graph kernels: GPU graph tests + heap walk vs level sweep timing; replay
# row-store A/B (lib vs lib_rm: only the slots an insert changed)
OUT=${1:-gpurun_out/r2k}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > "$OUT/graph_tests.log" 2>&1
rc=$?; echo "GRAPH TESTS rc=$rc"; tail -3 "$OUT/graph_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/level_bench.py 2000 > "$OUT/level_bench.log" 2>&1 || exit 1; cat "$OUT/level_bench.log"
for v in lib lib_rm lib lib_rm; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_$v.log" 2>&1 || exit 1; echo "$v: $(cut -c1-200 $OUT/kbench_$v.log)"
done
