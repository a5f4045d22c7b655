set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
export DTGPU_SEG=0
for k in ins friendsforever; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM \
    -d $O/$k -o run -f csv -- python -u tools/salu_probe.py $k 10000 > $O/$k.log 2>&1 || exit 1
  grep -h "replay" $O/$k.log | tail -1
done
