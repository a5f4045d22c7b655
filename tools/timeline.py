"""Kernel timeline of the last checkout pass in a rocprofv3 kernel trace: each dispatch's start and
end relative to the pass's first kernel, its grid and queue.  Usage: python tools/timeline.py CSV"""
import csv
import sys

PASS = ("prep_kernel", "chain_kernel", "walk_kernel", "plan_kernel", "replay_kernel", "combine_kernel", "cut_kernel",
        "fillBuffer")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    last = max(i for i, r in enumerate(rows) if "replay_kernel" in r["Kernel_Name"])
    end = last
    while end + 1 < len(rows) and "combine_kernel" in rows[end + 1]["Kernel_Name"]:
        end += 1
    i, body = last, False   # back to the previous pass's last replay / combine, past this pass's body
    while i > 0 and any(k in rows[i - 1]["Kernel_Name"] for k in PASS):
        name = rows[i - 1]["Kernel_Name"]
        end_kernel = "replay_kernel" in name or "combine_kernel" in name
        if end_kernel and body:
            break
        body = body or not (end_kernel or "fillBuffer" in name)
        i -= 1
    t0 = int(rows[i]["Start_Timestamp"])
    for r in rows[i:end + 1]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dtgpu::", "")
        print(f"{name[:52]:54s} {(int(r['Start_Timestamp']) - t0) / 1e6:8.3f} {(int(r['End_Timestamp']) - t0) / 1e6:8.3f} "
              f"grid={r['Grid_Size_X']:>7s} lds={r['LDS_Block_Size']:>6s} vgpr={r['VGPR_Count']} sgpr={r['SGPR_Count']} q={r['Queue_Id']}")


if __name__ == "__main__":
    main()
