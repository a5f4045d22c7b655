set -o pipefail
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 60 ./tools/occ_probe > $O/occ.log 2>&1; echo "occ rc=$?"; cat $O/occ.log
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
