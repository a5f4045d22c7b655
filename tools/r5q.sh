# kernel timeline of the last friendsforever x10000 pass (rocprofv3 kernel trace)
set -o pipefail
O=gpurun_out/r5q; rm -rf $O; mkdir -p $O
timeout -k 10 200 python -u tools/kbench.py ${1:-friendsforever} ${2:-10000} 3 || exit 1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -f csv -- python -u tools/kbench.py ${1:-friendsforever} ${2:-10000} 2 > $O/tr.log 2>&1 || exit 1
python tools/timeline.py $O/tr/run_kernel_trace.csv | tee $O/timeline.txt
