# quick GPU check used while iterating: the named test files, then one bench leg
# usage: bash tools/gpu_quick.sh OUTDIR "tests/test_a.py tests/test_b.py" [bench args...]
set -e
OUT=$1; TESTS=$2; shift 2
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > "$OUT/tests.log" 2>&1
if [ $# -gt 0 ]; then timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; fi
