set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
for v in lib lib_salu lib_valu lib_vmem lib_vmem2 lib_lds lib; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
