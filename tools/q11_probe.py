#!/usr/bin/env python3
"""Threshold <= 0 (quirk Q11) on one contig of the synthetic genome, both
directional buffers: K1q (parallel) against the exact whole-buffer replay
(UNIPEAK_Q11_REPLAY=1, a child process), timed beside the `-r 25` scan, and
the two record sets compared field by field (close_pos aside: the replay
names each closing add, K1q gives the rule).  One JSON line.

usage: python tools/q11_probe.py [CONTIG (default chr21)] [THR (default 0)]"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from unipeak_amd import capi  # noqa: E402


def run(name, thr, bw=50):
    rows = [l.split() for l in open(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
            if l.strip() and not l.startswith("#")]
    ci = [r[0] for r in rows].index(name)
    L = int(rows[ci][1])
    with capi.Lib(0) as g:
        g.set_params(bw, 1, 0.0029, region_thr=thr)
        for buf in (0, 1):
            u = g.add_unit(L, buffer_id=buf)
            g.synth(u, 0, 0, 1000, ci, buf, nondir=False, peaks=True)
        g.run()  # warm-up (allocations, capacities)
        ts = []
        for _ in range(3 if os.environ.get("UNIPEAK_Q11_REPLAY") != "1" else 1):
            t0 = time.perf_counter()
            n = g.run()
            ts.append(time.perf_counter() - t0)
        regs, cnt = g.regions(n)
        return L, min(ts), regs.copy(), cnt.copy()


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "chr21"
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    if os.environ.get("Q11_CHILD"):
        L, dt, regs, cnt = run(name, thr)
        np.savez(os.environ["Q11_CHILD"], regs=regs, cnt=cnt, dt=dt)
        return
    L, dt25, _, _ = run(name, 25.0)
    _, dtq, rq, cq = run(name, thr)
    out = os.path.join(ROOT, "gpurun_out", "q11_replay.npz")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    env = dict(os.environ, UNIPEAK_Q11_REPLAY="1", Q11_CHILD=out)
    subprocess.run([sys.executable, __file__, name, str(thr)], env=env, check=True, timeout=600)
    z = np.load(out)
    rr, cr, dtr = z["regs"], z["cnt"], float(z["dt"])
    fields = [f for f in rr.dtype.names if f != "close_pos"]
    same = len(rr) == len(rq) and all(
        rr[f].tobytes() == rq[f].tobytes() for f in fields) and cr.tobytes() == cq.tobytes()
    print(json.dumps({"contig": name, "bp": L, "region_thr": thr, "candidates": int(len(rq)),
                      "accepted": int(rq["accepted"].sum()), "ms_r25_scan": round(dt25 * 1e3, 3),
                      "ms_q11_parallel": round(dtq * 1e3, 3), "ms_q11_replay": round(dtr * 1e3, 1),
                      "parallel_over_r25": round(dtq / dt25, 2),
                      "records_identical_to_replay": bool(same)}), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
