set -o pipefail
O=gpurun_out/r5r; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -f csv -- python -u tools/kbench.py friendsforever 10000 3 > $O/tr.log 2>&1 || exit 1
grep kernel_ms $O/tr.log
python tools/timeline.py $O/tr/run_kernel_trace.csv
