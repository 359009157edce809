#!/usr/bin/env python3
"""Kernel timeline from a rocprofv3 --kernel-trace csv directory: the last
passes' kernels with start/end relative to the first shown, per queue, so the
overlap of consecutive passes is visible.  usage: timeline.py DIR [n]"""
import csv
import glob
import re
import sys

NAMES = [("scan_kernel<.*, 1>", "K1a"), ("xref_kernel", "K1x"), ("scan_kernel<.*, 2>", "K1b"),
         ("seg_count_head", "K2a"), ("seg_compact", "K2b"), ("stats_kernel", "K3")]


def short(n):
    for pat, s in NAMES:
        if re.search(pat, n):
            return s
    return n[:28]


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
                         short(r["Kernel_Name"])))
    rows.sort()
    rows = [r for r in rows if r[3] in {s for _, s in NAMES}]
    tail = rows[-n:]
    t0 = tail[0][0]
    k1a = [r for r in rows if r[3] == "K1a"]
    if len(k1a) > 3:
        per = [(k1a[i + 1][0] - k1a[i][0]) / 1e3 for i in range(len(k1a) - 6, len(k1a) - 1)]
        print("K1a start-to-start (us):", " ".join(f"{p:.1f}" for p in per))
    for s, e, q, name in tail:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{q} {name}")


if __name__ == "__main__":
    main()
