"""Short per-kernel summary (average µs, calls) of a rocprofv3 kernel_stats.csv."""
import csv
import re
import sys

short = [("scan_kernel<.*, 1>", "K1a"), ("scan_kernel<.*, 3>|k1a_fields_kernel", "K1a_fields"), ("scan_kernel<.*, 2>", "K1b"), ("seg_count_kernel", "K2a"), ("seg_count_head", "K2a+K0d"),
         ("seg_compact", "K2b"), ("stats_kernel", "K3"), ("stats1_kernel", "K3_one"), ("csum_units|pool_units|pct_units", "index"), ("head_detect|unit_last", "K0d")]
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for pat, name in short:
    for r in rows:
        if re.search(pat, r["Name"]):
            out.append(f"{name} {float(r['AverageNs']) / 1000:.1f}us x{r['Calls']}")
print(" ".join(out))
