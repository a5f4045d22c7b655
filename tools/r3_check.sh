#!/bin/bash
# Round-3 GPU iteration: parity tests, per-document cycle profile, batch kernel timing.
# Usage (inside gpurun): bash tools/r3_check.sh [tests|prof|bench|all] [pytest args...]
mkdir -p gpurun_out
what=${1:-all}; shift
rc=0
if [[ $what == tests || $what == all ]]; then
  timeout -k 10 400 python -u -m pytest ${@:-tests/test_gpu_parity.py tests/test_gpu_e2e.py} -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?; echo "TESTS $rc"; tail -4 gpurun_out/tests.log
  [[ $rc != 0 ]] && grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -20 && if [[ $what == ab ]]; then   # span vs per-item tracker on the same box
  for m in span item; do
    if [[ $m == item ]]; then export DTGPU_ITEM_REPLAY=1; else unset DTGPU_ITEM_REPLAY; fi
    echo "== $m"
    timeout -k 10 300 python -u tools/kbench.py friendsforever 1,10000 3 2>&1 | tee gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py git-makefile 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py node_nodecc 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
  done
fi
exit $rc
fi
if [[ $what == prof || $what == all ]]; then
  timeout -k 10 200 python -u tools/kprof.py friendsforever friendsforeverx4096 git-makefile node_nodecc > gpurun_out/kprof.log 2>&1
  rc=$?; echo "PROF $rc"; cat gpurun_out/kprof.log
  [[ $rc != 0 ]] && if [[ $what == ab ]]; then   # span vs per-item tracker on the same box
  for m in span item; do
    if [[ $m == item ]]; then export DTGPU_ITEM_REPLAY=1; else unset DTGPU_ITEM_REPLAY; fi
    echo "== $m"
    timeout -k 10 300 python -u tools/kbench.py friendsforever 1,10000 3 2>&1 | tee gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py git-makefile 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py node_nodecc 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
  done
fi
exit $rc
fi
if [[ $what == bench || $what == all ]]; then
  timeout -k 10 300 python -u tools/kbench.py friendsforever 1,10000 3 > gpurun_out/kbench.log 2>&1
  rc=$?; echo "BENCH $rc"; cat gpurun_out/kbench.log
fi
if [[ $what == ab ]]; then   # span vs per-item tracker on the same box
  for m in span item; do
    if [[ $m == item ]]; then export DTGPU_ITEM_REPLAY=1; else unset DTGPU_ITEM_REPLAY; fi
    echo "== $m"
    timeout -k 10 300 python -u tools/kbench.py friendsforever 1,10000 3 2>&1 | tee gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py git-makefile 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
    timeout -k 10 300 python -u tools/kbench.py node_nodecc 1 3 2>&1 | tee -a gpurun_out/kbench_$m.log
  done
fi
exit $rc
