#!/bin/bash
# Extra PMC passes (TA / TCP / TCC request mix) over the replay kernel; usage as tools/pmc.sh.
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p "$OUT"
CMD=("$@")
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run -f csv -- "${CMD[@]}" > "$OUT/$name.log" 2>&1
  echo "pass $name rc=$?"
}
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
pass ta TA_TA_BUSY_sum TA_BUSY_avr
pass tcp1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum
pass tcp2 TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
pass td TD_TD_BUSY_sum TD_BUSY_avr
pass tcc2 TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_REQ_sum TCC_BUSY_avr
pass sq3 SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES
