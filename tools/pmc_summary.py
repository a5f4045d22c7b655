"""Summarise rocprofv3 --pmc CSVs written by tools/pmc.sh: per-dispatch means of each counter
for the replay kernel, plus derived ratios."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "replay_kernel"
    agg = collections.defaultdict(float)
    nd = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern not in r.get("Kernel_Name", ""):
                continue
            nd[r["Counter_Name"]].add(r["Dispatch_Id"])
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    m = {k: v / max(1, len(nd[k])) for k, v in agg.items()}
    for k in sorted(m):
        print(f"{k:24s} {m[k]:.4g}")
    if "TCC_HIT_sum" in m:
        print(f"{'L2 hit rate':24s} {m['TCC_HIT_sum'] / max(1, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
    if "SQ_WAVE_CYCLES" in m:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            print(f"{k + ' frac':24s} {m[k] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_LDS_IDX_ACTIVE" in m:
        print(f"{'LDS bank-conflict rate':24s} {m['SQ_LDS_BANK_CONFLICT'] / max(1, m['SQ_LDS_IDX_ACTIVE']):.3f}")


if __name__ == "__main__":
    main()
