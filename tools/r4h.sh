set -o pipefail
OUT=gpurun_out/r4h; mkdir -p $OUT; : > $OUT/level_prof3.log
bash tools/gpu_steps.sh $OUT tests -- tests/test_gpu_graph.py || exit 1
for v in 256 64; do
  echo "pts=$v" >> $OUT/level_prof3.log
  DTGPU_LVL_PROF=1 DTGPU_LVL_PTS_LDS=$v timeout -k 10 200 python -u tools/level_bench.py >> $OUT/level_prof3.log 2>&1 || exit 1
done
grep -v "lvlprof" $OUT/level_prof3.log; grep lvlprof $OUT/level_prof3.log | awk 'NR%3==1'
