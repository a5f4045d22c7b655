set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
bash tools/gpu_steps.sh $O tests || exit 1
for v in "DTGPU_FLAT=0" "DTGPU_FLAT_WAVES=8" "DTGPU_FLAT_WAVES=7" "DTGPU_FLAT_WAVES=1"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 1,10000 3 || exit 1
done 2>&1 | tee $O/ab.log
