#!/bin/bash
# Evidence at HEAD (inside gpurun):  bash tools/evidence.sh OUTDIR
#   -m gpu tests, smoke(), bench line (+ rocprofv3 kernel stats, FETCH/WRITE -> traffic.json),
#   SQ/LDS/TCC counter passes for all checkout kernels, per-phase replay cycles, mixed workload.
OUT=${1:-gpurun_out/ev}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
cat "$OUT/smoke.log"
bash tools/bench_profile.sh "$OUT/bp" || exit 1
head -c 600 "$OUT/bp/bench.json"; echo
bash tools/pmc.sh "$OUT/pmc" python -u tools/kbench.py friendsforever 10000 1 || exit 1
timeout -k 10 200 python -u tools/kprof.py friendsforever friendsforeverx4096 git-makefile node_nodecc > "$OUT/kprof.log" 2>&1
timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/mixed.json" 2> "$OUT/mixed.err"
timeout -k 10 300 python -u bench.py --workload synth --distinct 1024 --docs 20000 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/synth.json" 2> "$OUT/synth.err"
echo done
