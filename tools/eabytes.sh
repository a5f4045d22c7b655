#!/bin/bash
# Memory-side bytes per kernel from the L2's EA request counters split by size (two rocprofv3
# passes: reads by 32/64/128-B request, writes by 32/64-B request) -- exact where FETCH_SIZE is
# not (it tallies a 128-B read as 64 B on gfx950, profiles/r2_calib).
#   bash tools/eabytes.sh OUTDIR CMD...   then   python tools/eabytes.py OUTDIR
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/rd" -o run -f csv -- "$@" > "$OUT/rd.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_sum -d "$OUT/wr" -o run -f csv -- "$@" > "$OUT/wr.log" 2>&1 || exit 1
echo "eabytes ok"
