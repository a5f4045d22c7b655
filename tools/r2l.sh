#!/bin/bash
# exec-mask-free loads in the replay (lib) vs HEAD (lib_old): GPU tests, kernel times, SALU counts
OUT=${1:-gpurun_out/r2l}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "ALL TESTS rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit 1
fi
for v in lib lib_old lib lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 120 python -u tools/kbench.py friendsforever 10000 3 > "$OUT/kbench_$v.log" 2>&1 || exit 1; echo "$v: $(cut -c1-200 $OUT/kbench_$v.log)"
done
for v in lib lib_old; do
  DTGPU_LIB_DIR=$v timeout -k 10 200 python -u tools/kprof.py friendsforever git-makefile node_nodecc > "$OUT/kprof_$v.log" 2>&1 || exit 1; echo "== $v"; cut -c1-120 "$OUT/kprof_$v.log"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for v in lib lib_old; do
  DTGPU_LIB_DIR=$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAVES -d "$OUT/sq_$v" -o run -f csv -- python3 tools/kbench.py friendsforever 10000 1 > "$OUT/sq_$v.log" 2>&1 || exit 1
  python3 - "$OUT/sq_$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
last = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "replay_kernel<true" not in k and "plan_kernel_1" not in k:
        continue
    last.setdefault(k, collections.OrderedDict())
    last[k][(r["Dispatch_Id"], r["Counter_Name"])] = float(r["Counter_Value"])
for k, d in last.items():
    disp = max(int(x[0]) for x in d)
    vals = {c: v for (di, c), v in d.items() if int(di) == disp}
    print(sys.argv[1].split("/")[-1], k[:40], {c: f"{v:.3e}" for c, v in sorted(vals.items())})
PY
done
