set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
for v in "DTGPU_PIPE=1" "DTGPU_PIPE=2 DTGPU_PIPE_FIRST=70" "DTGPU_PIPE=2 DTGPU_PIPE_FIRST=70 DTGPU_PIPE_PRIO=1" "DTGPU_PIPE=2 DTGPU_PIPE_FIRST=85 DTGPU_PIPE_PRIO=1" "DTGPU_PIPE=2 DTGPU_PIPE_PRIO=1"; do
  echo "-- $v"; env $v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
