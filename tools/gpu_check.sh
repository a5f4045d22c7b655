#!/bin/bash
# Standard GPU validation call: parity tests, per-document cycle profile, batch kernel timing.
# Usage (inside gpurun): bash tools/gpu_check.sh [kbench counts]
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "TESTS $?"
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u tools/kprof.py friendsforever friendsforeverx4096 git-makefile node_nodecc > gpurun_out/kprof.log 2>&1
echo "PROF $?"
timeout -k 10 300 python -u tools/kbench.py friendsforever ${1:-1,2048,4096,10000} 3 > gpurun_out/kbench.log 2>&1 && timeout -k 10 300 python -u tools/kbench.py synth:256 ${2:-1,4096,20000} 3 >> gpurun_out/kbench.log 2>&1
echo "BENCH $?"
