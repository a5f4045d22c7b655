set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT
bash tools/gpu_steps.sh $OUT tests || exit 1
LIBS="lib_base lib lib_w7 lib_w8 lib_pw8" bash tools/gpu_steps.sh $OUT ab || exit 1
