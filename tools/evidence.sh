#!/bin/bash
# Evidence at HEAD (inside gpurun):  bash tools/evidence.sh OUTDIR
#   -m gpu tests, smoke(), bench line (+ rocprofv3 kernel stats, FETCH/WRITE -> traffic.json),
#   the pass's kernel timeline, kbench of the three .dt files, mixed and configs[3] workloads.
OUT=${1:-gpurun_out/ev}   # SKIP_TESTS / SKIP_BP: leave those steps out
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
cat "$OUT/smoke.log"
fi
if [ -z "$SKIP_BP" ]; then
bash tools/bench_profile.sh "$OUT/bp" || exit 1
head -c 600 "$OUT/bp/bench.json"; echo
python tools/timeline.py "$OUT/bp/trace/run_kernel_trace.csv" > "$OUT/timeline.txt" || exit 1
fi
for t in friendsforever:1,10000 git-makefile:1 node_nodecc:1; do
  timeout -k 10 200 python -u tools/kbench.py ${t%%:*} ${t##*:} 3 || exit 1
done > "$OUT/kbench.log" 2>&1
cat "$OUT/kbench.log"
timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/mixed.json" 2> "$OUT/mixed.err" || exit 1
head -c 400 "$OUT/mixed.json"; echo
bash tools/bench_profile.sh "$OUT/lin" --workload linear --docs 2000 --steps 10 --warmup 2 || exit 1
head -c 400 "$OUT/lin/bench.json"; echo
DTGPU_STAGE_PROF=1 timeout -k 10 200 python -u tools/stage_probe.py friendsforever 10000 > "$OUT/stage_probe.log" 2>&1 || exit 1
tail -1 "$OUT/stage_probe.log"
timeout -k 10 500 python -u bench.py --workload synth --distinct 65536 --docs 125000 --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-encode > "$OUT/synth_125k.json" 2> "$OUT/synth_125k.err" || exit 1
head -c 400 "$OUT/synth_125k.json"; echo
echo done
