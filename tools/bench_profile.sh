#!/bin/bash
# Round-end evidence on the GPU box: bench JSON line, rocprofv3 kernel-trace stats of the same
# command, and FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) for the roofline traffic.
# Usage (inside gpurun): bash tools/bench_profile.sh OUTDIR [bench args...]
OUT=$1; shift
ARGS=("$@")
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py "${ARGS[@]}" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench rc=$?"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- python -u bench.py "${ARGS[@]}" --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/trace.log" 2>&1
echo "trace rc=$?"
# (DTGPU_PASS_MARK: every pass opens with a marker kernel, so tools/traffic.py sums exactly the
# last pass; --no-decode --no-encode: nothing runs after it)
DTGPU_PASS_MARK=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -f csv -- python -u bench.py "${ARGS[@]}" --no-cpu-baseline --no-decode --no-encode --steps 1 --warmup 1 > "$OUT/fetch.log" 2>&1
echo "fetch rc=$?"
DTGPU_PASS_MARK=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -f csv -- python -u bench.py "${ARGS[@]}" --no-cpu-baseline --no-decode --no-encode --steps 1 --warmup 1 > "$OUT/write.log" 2>&1
echo "write rc=$?"
python tools/traffic.py "$OUT/fetch" "$OUT/write" "$OUT/traffic.json" > /dev/null && echo "traffic ok"
