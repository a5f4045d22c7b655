#!/bin/bash
# GPU call: tests, bench line, read-width calibration, SQ counter passes on the replay (10k ff)
OUT=${1:-gpurun_out/r2c}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/wf" -o run -f csv -- ./tools/wprobe > "$OUT/wf.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum -d "$OUT/wr" -o run -f csv -- ./tools/wprobe > "$OUT/wr.log" 2>&1 || exit 1
bash tools/pmc.sh "$OUT/pmc" python -u tools/kbench.py friendsforever 10000 1
