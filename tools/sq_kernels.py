#!/usr/bin/env python3
"""Mean SQ counters per launch for every kernel name in rocprofv3 --pmc
counter_collection csv directories, grouped by kernel family (K1a / K1b /
K3 by scan_kernel's mode argument, others by name).

usage: python tools/sq_kernels.py DIR [DIR ...]   (prints JSON)"""
import csv
import glob
import json
import re
import sys


def family(name):
    m = re.search(r"scan_kernel<(.*)>", name)
    if m:
        mode = m.group(1).split(",")[-1].strip()
        return {"1": "K1a", "2": "K1b", "3": "K1a_fields"}.get(mode, "scan_mode" + mode)
    for pat, fam in (("k1a_fields_kernel", "K1a_fields"), ("stats1_kernel", "K3_one"), ("stats_kernel", "K3"), ("proc_runs", "K1q"), ("seg_", "K2"),
                     ("xref", "K1x")):
        if pat in name:
            return fam
    return name.split("(")[0][:40]


def main():
    acc = {}
    for d in sys.argv[1:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                c = acc.setdefault(family(r["Kernel_Name"]), {}).setdefault(r["Counter_Name"], {})
                c[r["Dispatch_Id"]] = c.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    res = {k: {n: round(sum(v.values()) / len(v), 1) for n, v in sorted(cs.items())}
           for k, cs in sorted(acc.items())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
