#!/usr/bin/env python3
"""Host cost per call of the pipelined pass API on a tiny genome (GPU time
negligible): set_record_target, set_timing, run_async, run_wait."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from unipeak_amd import capi  # noqa: E402

with capi.Lib(0) as g:
    g.set_params(50, 1, 0.003)
    for ci in range(4):
        u = g.add_unit(100_000, buffer_id=0)
        g.synth(u, 0, 0, 1000, ci, 0)
    g.set_params(50, 1, 0.0036, region_thr=25.0, kurt_thr=50.0, hit_thr=10.0)
    n0 = g.run()
    cap = n0 + 64
    bufs = [np.zeros(8 + cap * (capi.REGION_DTYPE.itemsize + 4) + 4096, np.uint8) for _ in range(6)]
    for b in bufs:
        g.host_register(b.ctypes.data, len(b))
    T = {"target": 0.0, "timing": 0.0, "async": 0.0, "wait": 0.0}
    N = 400
    for i in range(N + 20):
        t0 = time.perf_counter()
        g.set_record_target(bufs[i % 6].ctypes.data, cap)
        t1 = time.perf_counter()
        g.set_timing(1)
        t2 = time.perf_counter()
        g.run_async()
        t3 = time.perf_counter()
        if i >= 2:
            g.run_wait()
        t4 = time.perf_counter()
        if i >= 20:
            T["target"] += t1 - t0
            T["timing"] += t2 - t1
            T["async"] += t3 - t2
            T["wait"] += t4 - t3
    g.run_wait()
    g.run_wait()
    print({k: round(v / N * 1e6, 1) for k, v in T.items()}, "us per call", flush=True)
