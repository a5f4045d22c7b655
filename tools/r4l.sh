set -o pipefail
OUT=gpurun_out/r4l; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_e2e.py -k "plan" > $OUT/t.log 2>&1; tail -2 $OUT/t.log
for v in lib lib_spec; do echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kprof.py --plan friendsforever friendsforeverx10000 git-makefile | cut -c1-160; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 1,10000 3 | cut -c1-200; done
