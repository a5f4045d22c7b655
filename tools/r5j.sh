set -o pipefail
O=gpurun_out/r5j; mkdir -p $O
for v in "DTGPU_FLAT_WAVES=8" "DTGPU_FLAT_WAVES=7" "DTGPU_FLAT_WAVES=1" "DTGPU_LIB_DIR=lib_base DTGPU_FLAT_WAVES=8"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
