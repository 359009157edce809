#!/usr/bin/env python3
"""Region-length and exact-work statistics of the bench workload (hg19, one
directional sample, synthetic): what K1b / K3 latency depends on."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from unipeak_amd import capi, shard  # noqa: E402

contigs = bench.load_table(["hg19"])
lens = [L for _, L in contigs]
units, owner, mine = shard.plan(lens, nondir=False, world=1)
g = capi.Lib(0)
g.set_params(50, 1, 0.0029)
tags = 0
for k in mine[0]:
    ci, buf = units[k]
    u = g.add_unit(lens[ci], buffer_id=buf)
    g.synth(u, 0, 0, 1000, ci, buf)
    tags += g.tag_total(u, 0, 0)
g.set_params(50, 1, tags / sum(lens) / 2, region_thr=25.0, kurt_thr=50.0, hit_thr=10.0)
n = g.run()
r, c = g.regions(n)
ln = (r["right"].astype(np.int64) - r["left"] + 1)
print("regions", n, "len mean", ln.mean(), "p50", np.percentile(ln, 50), "p99", np.percentile(ln, 99),
      "max", ln.max(), "known peaks", None)
print("words per region p99", np.percentile((ln + 63) // 64, 99), "max", ((ln + 63) // 64).max())
print("timings", g.timings())
g.close()
cnt = c[:, 0].astype(np.int64)
m = (len(cnt) + 63) // 64
pad = np.zeros(m * 64, np.int64)
pad[:len(cnt)] = cnt
g = pad.reshape(m, 64)
print("count per region mean", cnt.mean(), "p99", np.percentile(cnt, 99), "max", cnt.max())
print("per 64-region wave: max count mean", g.max(1).mean(), "p50", np.percentile(g.max(1), 50),
      "p99", np.percentile(g.max(1), 99), "max", g.max(1).max(), "; waves with a region > 48 tags",
      int((g.max(1) > 48).sum()), "of", m, "; regions > 48 tags", int((cnt > 48).sum()))
