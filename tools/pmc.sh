#!/bin/bash
# PMC passes over the replay kernel (one rocprofv3 run per counter group, gfx950 slot limits):
#   bash tools/pmc.sh OUTDIR CMD...     e.g. bash tools/pmc.sh gpurun_out/pmc python tools/kbench.py friendsforever 4096 1
# Writes OUTDIR/<pass>/..._counter_collection.csv per pass.
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p "$OUT"
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- "${CMD[@]}" > "$OUT/$name.log" 2>&1
  echo "pass $name rc=$?"
}
CMD=("$@")
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pass sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
