#!/bin/bash
# Counter calibration + replay baseline (inside gpurun):  bash tools/calib.sh OUTDIR
# 1. tools/wprobe under WRITE_SIZE / FETCH_SIZE / TCC request passes (known byte counts per shape)
# 2. replay kernel request mix (TCP->TCC reads / writes / atomics) for 10k friendsforever
OUT=${1:-gpurun_out/calib}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
set -o pipefail
timeout -k 10 60 ./tools/wprobe > "$OUT/wprobe.txt" 2>&1 || { echo "wprobe failed"; exit 1; }
pass() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- ./tools/wprobe > "$OUT/$name.log" 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass w WRITE_SIZE && pass f FETCH_SIZE && pass ea TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_REQ_sum \
  && pass tcp TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum || exit 1
rpass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- python -u tools/kbench.py friendsforever 10000 1 > "$OUT/$name.log" 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
rpass rtcp TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum \
  && rpass rea TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
