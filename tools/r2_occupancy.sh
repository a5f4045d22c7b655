set -o pipefail
bash tools/r2_check.sh gpurun_out/r2b || exit 1
for pad in 1704 3752; do DTGPU_LDS_PAD=$pad timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > gpurun_out/r2b/kbench_pad$pad.log 2>&1 || exit 1; cat gpurun_out/r2b/kbench_pad$pad.log; done
