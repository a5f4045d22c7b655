#!/bin/bash
# PC sampling of one kbench run (inside gpurun): bash tools/pcsamp.sh OUTDIR METHOD DOC COUNT
# METHOD stochastic (cycles interval, stall reasons) or host_trap (time interval, us).
OUT=${1:?outdir}; M=${2:-stochastic}; DOC=${3:-node_nodecc}; N=${4:-1}
mkdir -p "$OUT"
timeout -k 10 90 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || { echo "list rc=$?"; exit 1; }
grep -iE "pc_sampling|method|unit|interval" "$OUT/avail.txt" | head -20
grep -qi "$M" "$OUT/avail.txt" || { echo "no $M pc sampling on this agent"; exit 0; }
if [[ $M == stochastic ]]; then U=cycles; I=${PCS_INTERVAL:-65536}; else U=time; I=${PCS_INTERVAL:-50}; fi
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
  --pc-sampling-interval $I -d "$OUT/pcs" -o run --output-format csv -- python3 -u tools/kbench.py $DOC $N 1 \
  > "$OUT/pcs.log" 2>&1
rc=$?; tail -5 "$OUT/pcs.log"; ls -la "$OUT"/pcs/* 2>/dev/null | head; exit $rc
