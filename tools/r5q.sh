set -o pipefail
O=gpurun_out/r5q; mkdir -p $O
for v in "DTGPU_PRIO=1" "DTGPU_LIB_DIR=lib_ramp" "DTGPU_PRIO=1" "DTGPU_LIB_DIR=lib_ramp"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
