set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_e2e.py tests/test_gpu_mixed.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -1 $O/t.log; [ $rc = 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for v in "X=1" "DTGPU_SEG_LATE=0"; do
echo "-- $v"
env $v timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -f csv -- python -u tools/kbench.py friendsforever 10000 3 > $O/tr.log 2>&1 || exit 1
grep kernel_ms $O/tr.log
python tools/timeline.py $O/tr/run_kernel_trace.csv
rm -rf $O/tr
done
