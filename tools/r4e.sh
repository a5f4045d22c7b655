set -o pipefail
OUT=gpurun_out/r4e; mkdir -p $OUT
: > $OUT/ldspad.log
for pad in 0 1800 3800 7000 14000; do
  echo "pad=$pad" >> $OUT/ldspad.log
  DTGPU_LDS_PAD=$pad timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 2 >> $OUT/ldspad.log 2>&1 || exit 1
done
cat $OUT/ldspad.log
