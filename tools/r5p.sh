set -o pipefail
O=gpurun_out/r5p; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc = 0 ] || exit 1
for t in friendsforever friendsforever; do
  timeout -k 10 200 python -u tools/kbench.py $t 10000 3 || exit 1
done 2>&1 | tee $O/ab.log
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -f csv -- python -u tools/kbench.py friendsforever 10000 1 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -f csv -- python -u tools/kbench.py friendsforever 10000 1 > $O/write.log 2>&1 || exit 1
python tools/traffic.py $O/fetch $O/write $O/traffic.json > /dev/null && echo traffic ok
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run -f csv -- python -u tools/kbench.py friendsforever 10000 2 > $O/tr.log 2>&1 || exit 1
python tools/timeline.py $O/tr/run_kernel_trace.csv | tee $O/timeline.txt
