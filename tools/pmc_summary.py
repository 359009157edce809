#!/usr/bin/env python3
"""Average PMC counters per kernel from rocprofv3 sqlite outputs under a
directory (tools/gpu_pmc.sh).  usage: pmc_summary.py DIR [kernel-substr ...]"""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    keys = sys.argv[2:] or ["scan_kernel", "stats_kernel"]
    agg = defaultdict(lambda: defaultdict(list))
    for db in glob.glob(f"{root}/**/*.db", recursive=True):
        con = sqlite3.connect(db)
        try:
            q = """select ks.kernel_name, ip.name, kd.id, sum(pe.value) from rocpd_pmc_event pe
                   join rocpd_info_pmc ip on pe.pmc_id = ip.id
                   join rocpd_event ev on pe.event_id = ev.id
                   join rocpd_kernel_dispatch kd on kd.event_id = ev.id
                   join rocpd_info_kernel_symbol ks on kd.kernel_id = ks.id
                   group by kd.id, ip.name"""
            for kname, cname, _, v in con.execute(q):
                for k in keys:
                    if k in kname:
                        agg[k][cname].append(v)
        except sqlite3.Error:
            pass
    for k, d in agg.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"  {c:22s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
