#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), corrected as
/opt/skills/guides/MI355X_MICROARCH.md's HBM section prescribes: both are in
KiB, and FETCH_SIZE counts half of a coalesced streaming read on gfx950, so
read bytes = 2 * FETCH_SIZE * 1024.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTRING ALG_BYTES_PER_LAUNCH [OUT.json]
"""
import csv
import glob
import json
import os
import sys


def read_counter(d, name, kernel):
    vals = []
    for p in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(p) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == name and kernel in row["Kernel_Name"]:
                    vals.append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    vals.sort()
    return [v for _, v in vals]


def main():
    fetch_dir, write_dir, kernel, alg = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    fetch = read_counter(fetch_dir, "FETCH_SIZE", kernel)
    write = read_counter(write_dir, "WRITE_SIZE", kernel)
    if not fetch or not write:
        sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for kernel '{kernel}'")
    n = min(len(fetch), len(write))
    launches = []
    for f, w in zip(fetch[:n], write[:n]):
        rd, wr = 2.0 * f * 1024.0, w * 1024.0
        launches.append({"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_read_bytes": rd,
                         "hbm_write_bytes": wr, "traffic_bytes": rd + wr})
    per = sum(l["traffic_bytes"] for l in launches) / n
    res = {"kernel": kernel,
           "note": "KiB counters; gfx950 FETCH_SIZE counts 1/2 of a wide streaming read "
                   "(MI355X_MICROARCH.md HBM section): read bytes = 2 x FETCH_SIZE x 1024",
           "launches": launches, "traffic_bytes_per_launch": per,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": per / alg}
    out = json.dumps(res, indent=1)
    if len(sys.argv) > 5:
        with open(sys.argv[5], "w") as f:
            f.write(out)
    print(json.dumps({k: v for k, v in res.items() if k != "launches"}))


if __name__ == "__main__":
    main()
