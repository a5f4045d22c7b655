set -o pipefail
OUT=gpurun_out/r4w; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_mixed.py > $OUT/t.log 2>&1; rc=$?; tail -2 $OUT/t.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/t.log | head -20; exit 1; }
timeout -k 10 200 python -u tools/kbench.py friendsforever 1,10000 3 | cut -c1-200
