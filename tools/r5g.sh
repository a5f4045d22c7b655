set -o pipefail
O=gpurun_out/r5g; mkdir -p $O
DTGPU_LIB_DIR=lib_clock timeout -k 10 200 python -u tools/clock_probe.py --units friendsforever 10000 2>&1 | tee $O/units.log
DTGPU_LIB_DIR=lib_clock timeout -k 10 200 python -u tools/clock_probe.py --units friendsforever 8192 2>&1 | tee -a $O/units.log
DTGPU_LIB_DIR=lib_clock timeout -k 10 200 python -u tools/clock_probe.py friendsforever 8192 2>&1 | tee -a $O/units.log
