set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
for v in "DTGPU_LIB_DIR=lib" "DTGPU_LIB_DIR=lib_nocache" "DTGPU_LIB_DIR=lib DTGPU_FLAT_WAVES=7" "DTGPU_LIB_DIR=lib_nocache DTGPU_FLAT_WAVES=7" "DTGPU_LIB_DIR=lib" "DTGPU_LIB_DIR=lib_nocache"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
