set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
bash tools/gpu_steps.sh $O tests || exit 1
for v in lib_base lib lib_base lib; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
