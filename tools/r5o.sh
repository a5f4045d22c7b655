set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_parity.py tests/test_gpu_mixed.py tests/test_gpu_segments.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc = 0 ] || exit 1
for v in lib_base lib lib_base lib; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
