set -o pipefail
OUT=gpurun_out/r4c; mkdir -p $OUT
bash tools/gpu_steps.sh $OUT tests -- tests/test_gpu_parity.py tests/test_gpu_e2e.py tests/test_gpu_mixed.py tests/test_gpu_graph.py -m gpu
LIBS="lib_base lib_nocache lib_nocache_w6 lib lib_w6" bash tools/gpu_steps.sh $OUT ab || exit 1
(export DTGPU_HELP_TIER=4; timeout -k 10 200 python -u tools/kbench.py git-makefile 1 3 && timeout -k 10 200 python -u tools/kbench.py node_nodecc 1 3) > $OUT/kbench_nohelp.log 2>&1; cat $OUT/kbench_nohelp.log
KPROF_DOCS="friendsforever node_nodecc" bash tools/gpu_steps.sh $OUT kprof || exit 1
timeout -k 10 300 python -u tools/addbench.py node_nodecc 2048 > $OUT/addbench.log 2>&1; timeout -k 10 200 python -u tools/addbench.py git-makefile 4096 >> $OUT/addbench.log 2>&1; cat $OUT/addbench.log
