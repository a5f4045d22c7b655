# FF + hardening checks on the GPU box: bash tools/ff_steps.sh OUTDIR [pytest files...]
set -o pipefail
OUT=${1:-gpurun_out/r6_ff}; shift
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${@:-tests/test_gpu_ff.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -25 $OUT/tests.log
[ $rc = 0 ] || exit $rc
for t in automerge-paper rustcode seph-blog1 sveltecomponent friendsforever_flat; do
  timeout -k 10 120 python -u tools/kbench.py $t 1,1000 5 || exit 1
done 2>&1 | tee $OUT/kbench.log
