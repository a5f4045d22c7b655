"""HBM traffic per checkout pass from rocprofv3 PMC runs (FETCH_SIZE and WRITE_SIZE in separate
passes, MI355X_MICROARCH.md HBM section): for each checkout kernel the last dispatch of the run
is taken (earlier ones are the staging sizing pass and warmups); bytes = 2 * FETCH_SIZE (gfx950
reports half of a wide read) + WRITE_SIZE, both in KiB.
Usage: python tools/traffic.py FETCH_DIR WRITE_DIR OUT.json"""
import csv
import glob
import json
import os
import sys

KERNELS = ("prep_kernel", "plan_kernel", "replay_kernel")


def last_per_kernel(d, counter):
    last = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or not any(k in r["Kernel_Name"] for k in KERNELS):
                continue
            key = r["Kernel_Name"]
            did = int(r["Dispatch_Id"])
            prev = last.get(key)
            if prev is None or did > prev[0]:
                last[key] = (did, 0.0)
            if last[key][0] == did:
                last[key] = (did, last[key][1] + float(r["Counter_Value"]))
    return {k: v[1] for k, v in last.items()}


def main():
    fetch = last_per_kernel(sys.argv[1], "FETCH_SIZE")
    write = last_per_kernel(sys.argv[2], "WRITE_SIZE")
    per = {k: {"fetch_kib": fetch.get(k, 0.0), "write_kib": write.get(k, 0.0)} for k in set(fetch) | set(write)}
    total = sum(2 * v["fetch_kib"] + v["write_kib"] for v in per.values()) * 1024
    out = {"hbm_bytes_per_pass": total, "per_kernel": per,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024, last dispatch of each kernel"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
