#!/usr/bin/env python3
"""Per-step GPU timeline of a bench run from a rocprofv3 kernel trace.

usage: python tools/timeline_stats.py <trace dir or csv> [last_steps (default 20)] [skip (default 3)]

For the last N K1a launches (the timed passes) prints: K1a durations, the
gap between one K1a's end and the next one's start, what kernels ran in
that gap, and the share of wall time in which 0 / 1 / 2+ kernels were
active.  One JSON object."""
import csv
import glob
import json
import os
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    if os.path.isdir(path):
        path = glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((s, e, name))
    rows.sort()

    def short(n):
        if "k1a_fields_kernel" in n:
            return "K1a"
        if "scan_kernel" in n:
            m = n.split(">")[0]
            return "K1a" if (m.endswith(", 1") or m.endswith(", 3")) else ("K1b" if m.endswith(", 2") else "K1?")
        for k, v in (("stats1_kernel", "K3"), ("stats_kernel", "K3"), ("seg_count", "K2a"), ("seg_compact", "K2b"), ("xref", "K1x"),
                     ("emulate", "K0"), ("head", "K0h"), ("fillBuffer", "fill"), ("copyBuffer", "copy")):
            if k in n:
                return v
        return n.split("(")[0][-24:]

    ev = [(s, e, short(n)) for s, e, n in rows]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 3  # bench's blocking passes after the timed region
    k1a_all = [x for x in ev if x[2] == "K1a"]
    k1a = k1a_all[len(k1a_all) - skip - last - 1:len(k1a_all) - skip]
    t0, t1 = k1a[0][0], k1a[-1][0]  # from the first K1a start to the last one's start: `last` whole steps
    win = [x for x in ev if x[1] > t0 and x[0] < t1]
    # concurrency profile
    pts = []
    for s, e, _ in win:
        pts.append((max(s, t0), 1))
        pts.append((min(e, t1), -1))
    pts.sort()
    cur, prev, busy = 0, t0, {0: 0, 1: 0, 2: 0}
    for t, d in pts:
        busy[min(cur, 2)] += t - prev
        cur += d
        prev = t
    busy[min(cur, 2)] += t1 - prev
    tot = t1 - t0
    gaps = []
    for a, b in zip(k1a[:-1], k1a[1:]):
        inside = [x[2] for x in ev if x[0] < b[0] and x[1] > a[1]]
        gaps.append({"gap_us": round((b[0] - a[1]) / 1e3, 1), "kernels": inside})
    per = {}
    for s, e, n in win:
        d = per.setdefault(n, [0, 0.0])
        d[0] += 1
        d[1] += (min(e, t1) - max(s, t0)) / 1e3
    print(json.dumps({
        "steps": last, "ms_per_step": round(tot / last / 1e6, 4),
        "k1a_us": [round((e - s) / 1e3, 1) for s, e, _ in k1a[:-1]],
        "k1a_mean_us": round(sum(e - s for s, e, _ in k1a[:-1]) / last / 1e3, 1),
        "gap_after_k1a": gaps[-8:],
        "gap_mean_us": round(sum(g["gap_us"] for g in gaps) / len(gaps), 1),
        "share_idle_1_2plus": [round(busy[k] / tot, 3) for k in (0, 1, 2)],
        "kernel_us_per_step": {k: [v[0] / last, round(v[1] / last, 1)] for k, v in sorted(per.items())},
    }, indent=1))


if __name__ == "__main__":
    main()
