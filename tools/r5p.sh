set -o pipefail
O=gpurun_out/r5p; mkdir -p $O
for v in lib lib_nocb lib_nopf lib_nocbpf lib lib_nocb lib_nopf lib_nocbpf; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
