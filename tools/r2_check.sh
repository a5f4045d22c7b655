#!/bin/bash
# GPU validation + replay evidence in one call (inside gpurun):  bash tools/r2_check.sh OUTDIR [skip-tests]
#   parity tests, kernel timing (kbench), per-phase cycles (kprof), and the replay's request mix /
#   HBM counters (one rocprofv3 pass per group) on 10k friendsforever documents.
OUT=${1:-gpurun_out/r2}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
if [ -z "$2" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 200 python -u tools/kbench.py friendsforever 1,4096,10000 3 > "$OUT/kbench.log" 2>&1 || { echo "kbench failed"; exit 1; }
cat "$OUT/kbench.log"
timeout -k 10 200 python -u tools/kprof.py friendsforever friendsforeverx4096 git-makefile node_nodecc > "$OUT/kprof.log" 2>&1 || { echo "kprof failed"; exit 1; }
cat "$OUT/kprof.log"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
rpass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- python -u tools/kbench.py friendsforever 10000 1 > "$OUT/$name.log" 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
rpass rtcp TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum \
  && rpass rea TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_REQ_sum \
  && rpass write WRITE_SIZE && rpass fetch FETCH_SIZE && rpass tcc TCC_HIT_sum TCC_MISS_sum
