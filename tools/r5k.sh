set -o pipefail
O=gpurun_out/r5k; mkdir -p $O
for v in lib_base lib lib_skipu lib_base lib lib_skipu; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
