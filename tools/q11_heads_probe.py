#!/usr/bin/env python3
"""Threshold <= 0 with head units: chr19-chr22 of the
synthetic genome plus a chrM-like contig carrying tags at positions 3 and 40,
both directional buffers, generated on the device.  Times up_run at -r 25
and at -r 0 (K1q + the exact chains around chrM), with the pass's own split
(K1q / K2 / K3 / host wall) at timing level 2.  One JSON line.

usage: python tools/q11_heads_probe.py [REPS (default 5)]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from unipeak_amd import capi  # noqa: E402

HG = ["chr19", "chr20", "chrM", "chr21", "chr22"]


def table():
    rows = [l.split() for l in open(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
            if l.strip() and not l.startswith("#")]
    names = [r[0] for r in rows]
    return [(n, int(rows[names.index(n)][1]), names.index(n)) for n in HG]


def run(thr, reps, bw=50):
    with capi.Lib(0) as g:
        g.set_params(bw, 1, 0.0029, region_thr=thr)
        bp = 0
        for buf in (0, 1):
            for name, L, ci in table():
                u = g.add_unit(L, buffer_id=buf)
                g.synth(u, 0, 0, 1000, ci, buf, nondir=False, peaks=True)
                if name == "chrM":  # head tags: position 1 is processed
                    g.scatter(u, 0, 0, np.array([3, 40], np.uint32), np.array([2, 1], np.uint32))
                bp += L
        g.run()  # warm-up (allocations, capacities)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            n = g.run()
            ts.append(time.perf_counter() - t0)
        g.set_timing(2)
        n = g.run()
        split = [round(x, 3) for x in g.timings()]
        regs, _ = g.regions(n)
        return bp, min(ts), split, regs.copy()


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    bp, t25, s25, r25 = run(25.0, reps)
    _, t0, s0, r0 = run(0.0, reps)
    chains = int((r0["close_pos"] < 0xFFFFFFFD).sum())
    print(json.dumps({"contigs": HG, "bp_both_buffers": bp, "ms_r25": round(t25 * 1e3, 3),
                      "ms_r0": round(t0 * 1e3, 3), "r0_over_r25": round(t0 / t25, 2),
                      "split_r25_k1_k2_k3_wall_k1b": s25, "split_r0_k1q_k2_k3_wall": s0,
                      "records_r25": int(len(r25)), "records_r0": int(len(r0)),
                      "records_r0_from_chains": chains}), flush=True)


if __name__ == "__main__":
    main()
