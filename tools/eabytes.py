"""Summarise tools/eabytes.sh: per kernel (last dispatch) read bytes = 32*RDREQ_32B + 64*RDREQ_64B
+ 128*RDREQ_128B and write bytes = 64*WRREQ_64B + 32*(WRREQ - WRREQ_64B); also the DRAM share of
the requests (the rest are served by the Infinity Cache).  python tools/eabytes.py OUTDIR [OUT.json]"""
import csv
import glob
import json
import os
import sys


def last(d):
    per = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k, did = r["Kernel_Name"], int(r["Dispatch_Id"])
            cur = per.get(k)
            if cur is None or did > cur[0]:
                per[k] = cur = (did, {})
            if cur[0] == did:
                cur[1][r["Counter_Name"]] = cur[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {k: v[1] for k, v in per.items()}


def main():
    root = sys.argv[1]
    rd, wr = last(os.path.join(root, "rd")), last(os.path.join(root, "wr"))
    out = {}
    for k in sorted(set(rd) | set(wr)):
        a, b = rd.get(k, {}), wr.get(k, {})
        rbytes = 32 * a.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * a.get("TCC_EA0_RDREQ_64B_sum", 0) + \
            128 * a.get("TCC_EA0_RDREQ_128B_sum", 0)
        wreq, w64 = b.get("TCC_EA0_WRREQ_sum", 0), b.get("TCC_EA0_WRREQ_64B_sum", 0)
        wbytes = 64 * w64 + 32 * (wreq - w64)
        out[k] = {"read_bytes": rbytes, "write_bytes": wbytes, "rd_requests": a.get("TCC_EA0_RDREQ_sum", 0),
                  "rd_req_split_32_64_128": [a.get("TCC_EA0_RDREQ_32B_sum", 0), a.get("TCC_EA0_RDREQ_64B_sum", 0),
                                             a.get("TCC_EA0_RDREQ_128B_sum", 0)],
                  "rd_dram_requests": b.get("TCC_EA0_RDREQ_DRAM_sum", 0), "wr_requests": wreq,
                  "wr_dram_requests": b.get("TCC_EA0_WRREQ_DRAM_sum", 0)}
        print(f"{k[:70]:70s} read {rbytes / 1e9:8.3f} GB write {wbytes / 1e9:8.3f} GB")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
