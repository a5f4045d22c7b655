#!/bin/bash
# GPU call: new tests first (verbose), then the whole -m gpu suite, synth + mixed kernel timings
OUT=${1:-gpurun_out/r2d}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_synth_merge.py tests/test_gpu_mixed.py tests/test_shard_gloo.py tests/test_ffi_crate.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/new_tests.log" 2>&1
rc=$?; echo "NEW TESTS rc=$rc"; tail -12 "$OUT/new_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/kbench.py synth:256 4096,20000 3 > "$OUT/kbench_synth.log" 2>&1; cat "$OUT/kbench_synth.log"
