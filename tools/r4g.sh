set -o pipefail
OUT=gpurun_out/r4g; mkdir -p $OUT
bash tools/gpu_steps.sh $OUT tests -- tests/test_gpu_graph.py || exit 1
: > $OUT/level_ab.log
for v in "1 256" "0 0" "0 256" "1 0" "1 1024"; do
  set -- $v
  echo "head=$1 pts=$2" >> $OUT/level_ab.log
  DTGPU_LVL_HEAD_LDS=$1 DTGPU_LVL_PTS_LDS=$2 timeout -k 10 200 python -u tools/level_bench.py >> $OUT/level_ab.log 2>&1 || exit 1
done
cat $OUT/level_ab.log
bash tools/pcsamp.sh $OUT/pcs stochastic node_nodecc 1
