set -o pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_e2e.py -x -q --timeout 240 > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
for v in lib_base lib lib_base lib; do
  echo "-- $v"; DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kbench.py friendsforever 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
export DTGPU_SEG=0
for k in ins friendsforever; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM \
    -d $O/$k -o run -f csv -- python -u tools/salu_probe.py $k 10000 > $O/$k.log 2>&1 || exit 1
  grep -h "replay" $O/$k.log | tail -1
done
