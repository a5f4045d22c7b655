#!/bin/bash
OUT=${1:-gpurun_out/r2i}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/kprof.py friendsforever git-makefile node_nodecc > "$OUT/kprof.log" 2>&1; cut -c1-250 "$OUT/kprof.log"
timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench.log" 2>&1; cat "$OUT/kbench.log"
timeout -k 10 300 python -u bench.py --workload mixed --docs 400 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/mixed.json" 2> "$OUT/mixed.err"; python -c "
import json; d=json.load(open('$OUT/mixed.json')); print('mixed', d['value']/1e6, 'M ops/s', d['roofline']['pass'], d['e2e']['decode_ms'])"
