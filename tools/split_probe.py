#!/usr/bin/env python3
"""Throughput probe: the bench genome split over K contexts on ONE GPU (each
its own stream, units LPT-split), passes pipelined per context, so one
context's latency-bound kernels (K1b/K2/K3) can overlap another's streaming
K1a.  Host record delivery, no merge.  usage: split_probe.py K [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (torch's HIP runtime first, tools/mix_probe.py)
import bench  # noqa: E402
from unipeak_amd import capi, shard  # noqa: E402

torch.cuda.set_device(0)
K = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
contigs = bench.load_table(["hg19"])
lens = [L for _, L in contigs]
units, owner, mine = shard.plan(lens, nondir=False, world=K)
gs = []
tags = 0
for r in range(K):
    g = capi.Lib(0)
    g.set_params(50, 1, 0.0029)
    for k in mine[r]:
        ci, buf = units[k]
        u = g.add_unit(lens[ci], buffer_id=buf)
        g.synth(u, 0, 0, 1000, ci, buf)
        tags += g.tag_total(u, 0, 0)
    gs.append(g)
bg = tags / (sum(lens) & 0xFFFFFFFF) / 2
for g in gs:
    g.set_params(50, 1, bg, region_thr=25.0, kurt_thr=50.0, hit_thr=10.0)
    g.set_timing(0)
    g.run()


def run(n):
    inflight = 0
    nreg = 0
    for i in range(n):
        for g in gs:
            g.run_async()
        inflight += 1
        if inflight == 2:
            for g in gs:
                nreg += g.run_wait()
            inflight -= 1
    while inflight:
        for g in gs:
            nreg += g.run_wait()
        inflight -= 1
    return nreg


run(3)
torch.cuda.synchronize()
t0 = time.perf_counter()
n = run(steps)
dt = (time.perf_counter() - t0) / steps
print(f"K={K} ms/step {dt * 1e3:.4f} Gbp/s {sum(lens) / dt / 1e9:.1f} regions/step {n / steps:.0f}", flush=True)
