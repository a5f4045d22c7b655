set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
for v in "DTGPU_FLAT_WAVES=8" "DTGPU_SEG_FAIR=0 DTGPU_SEG_OPS=2000" "DTGPU_SEG_FAIR=0 DTGPU_SEG_OPS=1350" "DTGPU_SEG_FAIR=0 DTGPU_SEG_OPS=1000" "DTGPU_SEG_FAIR=0 DTGPU_SEG_OPS=700"; do
  echo "-- $v"; env $v timeout -k 10 300 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
