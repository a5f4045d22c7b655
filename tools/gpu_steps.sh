#!/bin/bash
# One parameterised GPU call (run inside gpurun): bash tools/gpu_steps.sh OUTDIR step[,step...] [-- pytest args]
# Steps run in order; the first failing step ends the call (nothing further touches the GPU).
#   tests      pytest -m gpu (or the given pytest args)                      OUT/gpu_tests.log
#   smoke      __graft_entry__.smoke()                                       OUT/smoke.log
#   bench      bench.py line + rocprofv3 kernel stats + FETCH/WRITE passes   OUT/bp/ (tools/bench_profile.sh)
#   kbench     friendsforever 1 / 10k, git-makefile, node_nodecc kernel ms  OUT/kbench.log
#   kprof      per-document replay cycle profile (DTGPU_DEBUG=2)             OUT/kprof.log
#   ab         kbench for every build in $LIBS (DTGPU_LIB_DIR, tools/variant.sh builds them)
#   pmc        SQ / LDS / TCC counter passes on 10k friendsforever          OUT/pmc/ (tools/pmc.sh)
#   mixed      bench.py --workload mixed (configs[4])                         OUT/mixed.json
#   synth      bench.py --workload synth at $SYNTH_DOCS / $SYNTH_DISTINCT     OUT/synth.json
#   plan       planner cycle profile                                         OUT/plan.log
#   level      heap walk vs level-synchronous graph queries                 OUT/level.log
OUT=${1:?outdir}; STEPS=${2:?steps}; shift 2
[[ $1 == -- ]] && shift
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p "$OUT"
ok() { echo "== $1 rc=$2"; [[ $2 == 0 ]] || exit "$2"; }
kb() {   # kbench over the three benchmark files
  timeout -k 10 200 python -u tools/kbench.py friendsforever 1,10000 3 && \
  timeout -k 10 200 python -u tools/kbench.py git-makefile 1 3 && \
  timeout -k 10 200 python -u tools/kbench.py node_nodecc 1 3 && \
  if [[ -n $KB_SYNTH ]]; then timeout -k 10 300 python -u tools/kbench.py synth:$KB_SYNTH 1,20000 3; fi
}
for s in ${STEPS//,/ }; do
  case $s in
    tests)
      # a heartbeat line a minute: a slow test (the spawned multi-process ones on a cold box)
      # prints nothing until it ends
      ( while sleep 60; do echo "tests running: $(grep -c -E 'PASSED|FAILED' "$OUT/gpu_tests.log" 2>/dev/null) done"; done ) &
      hb=$!
      timeout -k 10 900 python -u -m pytest ${@:-tests -m gpu} -x -v --timeout 480 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1
      rc=$?; kill $hb 2>/dev/null; tail -3 "$OUT/gpu_tests.log"; [[ $rc != 0 ]] && grep -E "FAILED|Error" "$OUT/gpu_tests.log" | head -20
      ok tests $rc ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; cat "$OUT/smoke.log"; ok smoke $rc ;;
    bench)
      bash tools/bench_profile.sh "$OUT/bp"; rc=$?
      head -c 700 "$OUT/bp/bench.json"; echo; ok bench $rc ;;
    kbench)
      kb > "$OUT/kbench.log" 2>&1; rc=$?; cat "$OUT/kbench.log"; ok kbench $rc ;;
    kprof)
      timeout -k 10 300 python -u tools/kprof.py ${KPROF_DOCS:-friendsforever friendsforeverx4096 git-makefile node_nodecc} \
        > "$OUT/kprof.log" 2>&1
      rc=$?; cut -c1-400 "$OUT/kprof.log"; ok kprof $rc ;;
    ab)
      for v in ${LIBS:-lib}; do
        DTGPU_LIB_DIR=$v kb > "$OUT/kbench_${v}.log" 2>&1; rc=$?
        echo "-- $v"; cut -c1-220 "$OUT/kbench_${v}.log"; ok "ab $v" $rc
      done ;;
    pmc)
      bash tools/pmc.sh "$OUT/pmc" python -u tools/kbench.py friendsforever 10000 1; ok pmc $? ;;
    mixed)
      timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline \
        > "$OUT/mixed.json" 2> "$OUT/mixed.err"
      rc=$?; head -c 400 "$OUT/mixed.json"; echo; ok mixed $rc ;;
    synth)
      timeout -k 10 900 python -u bench.py --workload synth --distinct ${SYNTH_DISTINCT:-1024} \
        --docs ${SYNTH_DOCS:-20000} --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/synth.json" 2> "$OUT/synth.err"
      rc=$?; head -c 400 "$OUT/synth.json"; echo; tail -3 "$OUT/synth.err"; ok synth $rc ;;
    level)
      timeout -k 10 300 python -u tools/level_bench.py > "$OUT/level.log" 2>&1
      rc=$?; cat "$OUT/level.log"; ok level $rc ;;
    plan)
      timeout -k 10 200 python -u tools/kprof.py --plan friendsforever friendsforeverx10000 git-makefile node_nodecc \
        > "$OUT/plan.log" 2>&1
      rc=$?; cat "$OUT/plan.log"; ok plan $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
