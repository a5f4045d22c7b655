set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_e2e.py tests/test_gpu_mixed.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -15 $O/t.log; [ $rc = 0 ] || exit 1
for v in "X=1" "DTGPU_SEG_LATE=0"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
