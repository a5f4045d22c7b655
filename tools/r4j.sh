set -o pipefail
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_e2e.py -k "plan or staged or golden or large" > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; exit 1; }
for v in 1 0; do echo "split=$v"; DTGPU_PLAN_SPLIT=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 1,10000 3 | cut -c1-200; DTGPU_PLAN_SPLIT=$v timeout -k 10 200 python -u tools/kbench.py git-makefile 1 2 | cut -c1-200; DTGPU_PLAN_SPLIT=$v timeout -k 10 200 python -u tools/kbench.py node_nodecc 1 2 | cut -c1-200; done
