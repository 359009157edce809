#!/usr/bin/env python3
"""K3 time with records delivered into mapped pinned host memory (default)
vs a device buffer (up_set_record_target with a device pointer): does writing
the records over PCIe bound K3?  hg19 bench workload, one context."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from unipeak_amd import capi, shard  # noqa: E402

torch.cuda.set_device(0)
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
g.set_params(50, 1, tags / (sum(lens) & 0xFFFFFFFF) / 2, region_thr=25.0, kurt_thr=50.0, hit_thr=10.0)
g.set_timing(2)
n = g.run()
cap = int(n * 1.25) + 64


def measure(label, reps=20):
    t = []
    for _ in range(reps):
        g.run()
        t.append(g.timings())
    t = np.array(t[2:])
    print(f"{label}: K1 {t[:, 0].mean():.4f} K2 {t[:, 1].mean():.4f} K3 {t[:, 2].mean():.4f} ms", flush=True)


measure("host (mapped pinned)")
buf = torch.empty(8 + cap * (capi.REGION_DTYPE.itemsize + 4), dtype=torch.uint8, device="cuda:0")
torch.cuda.synchronize()
g.set_record_target(buf.data_ptr(), cap)
measure("device buffer")
g.set_record_target(0, 0)
measure("host again")
