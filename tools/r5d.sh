set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
bash tools/pmc3.sh $O/flat8 python -u tools/kbench.py friendsforever 10000 1 || exit 1
DTGPU_FLAT=0 bash tools/pmc3.sh $O/lds python -u tools/kbench.py friendsforever 10000 1 || exit 1
python tools/pmc_summary.py $O/flat8 > $O/flat8.txt; python tools/pmc_summary.py $O/lds > $O/lds.txt
paste $O/flat8.txt $O/lds.txt
