#!/usr/bin/env python3
"""Mean SQ counters per launch of K1a / K1b / K3 from rocprofv3 --pmc
counter_collection csv directories (one pass of <= 8 SQ counters each).

usage: python tools/sq_summary.py OUT.json NOTE DIR [DIR ...]"""
import csv
import glob
import json
import re
import sys

KERNELS = [("K1a", r"scan_kernel<1, 0, false, false, 1>"), ("K1b", r"scan_kernel<1, 0, false, false, 2>"),
           ("K3", r"stats_kernel<1, 0, false>")]


def main():
    out, note, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc = {k: {} for k, _ in KERNELS}
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                for k, pat in KERNELS:
                    if re.search(re.escape(pat), r["Kernel_Name"]):
                        c = acc[k].setdefault(r["Counter_Name"], {})
                        c[r["Dispatch_Id"]] = c.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    res = {"note": note}
    for k, _ in KERNELS:
        res[k] = {n: round(sum(v.values()) / len(v), 1) for n, v in sorted(acc[k].items()) if v}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k].get("SQ_INSTS_VALU") for k, _ in KERNELS}))


if __name__ == "__main__":
    main()
