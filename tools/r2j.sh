#!/bin/bash
# A/B: cached-block position shortcut (lib) vs the previous build (lib_old) vs masked row
# stores (lib_rm): GPU tests, kernel times, per-phase single-document cycles, replay traffic.
OUT=${1:-gpurun_out/r2j}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
for v in lib lib_old lib_rm lib lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_$v.log" 2>&1 || exit 1; echo "$v: $(cut -c1-200 $OUT/kbench_$v.log)"
done
for v in lib lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kprof.py friendsforever git-makefile node_nodecc > "$OUT/kprof_$v.log" 2>&1 || exit 1; echo "== $v"; cut -c1-200 "$OUT/kprof_$v.log"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for v in lib lib_rm; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DTGPU_LIB_DIR=$v timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/pmc_${v}_$c" -o run -f csv -- python3 tools/kbench.py friendsforever 10000 1 > "$OUT/pmc_${v}_$c.log" 2>&1 || exit 1
  done
  python3 tools/traffic.py "$OUT/pmc_${v}_FETCH_SIZE" "$OUT/pmc_${v}_WRITE_SIZE" "$OUT/traffic_$v.json" && echo "traffic $v" && cat "$OUT/traffic_$v.json"
done
