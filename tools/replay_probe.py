#!/usr/bin/env python3
"""Time the exact whole-buffer replay against the parallel
scan on one contig of the synthetic genome: `-r 25` (parallel scan), `-r 0`
(quirk Q11 live: K1q), `-b 150` / `-b 300` / `-b 511` (parallel, NH = 3 / 5 /
8) and `-b 600` / `-b 2000` (the whole-buffer replay: wider than the
register halo).  Blocking up_run, both directional buffers of
the contig, one line of JSON per configuration.

usage: python tools/replay_probe.py [CONTIG (default chr21)]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from unipeak_amd import capi  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "chr21"
    rows = [l.split() for l in open(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
            if l.strip() and not l.startswith("#")]
    ci = [r[0] for r in rows].index(name)
    L = int(rows[ci][1])
    for bw, thr in ((50, 25.0), (50, 0.0), (150, 25.0), (300, 25.0), (511, 25.0), (300, 0.0),
                    (600, 25.0), (2000, 25.0)):
        with capi.Lib(0) as g:
            g.set_params(bw, 1, 0.0029, region_thr=thr)
            for buf in (0, 1):
                u = g.add_unit(L, buffer_id=buf)
                g.synth(u, 0, 0, 1000, ci, buf, nondir=False, peaks=True)
            if bw <= 511:
                g.run()  # warm-up (allocations; the replay grows its capacities itself)
            t0 = time.perf_counter()
            n = g.run()
            dt = time.perf_counter() - t0
            regs, _ = g.regions(n)
            print(json.dumps({"contig": name, "bp": L, "bw": bw, "region_thr": thr,
                              "path": ("wide" if thr > 0 else "replay") if bw > 511 else ("K1q" if thr <= 0 else "scan"), "ms": round(dt * 1e3, 3),
                              "gbps": round(L / dt / 1e9, 3), "candidates": int(n),
                              "accepted": int(regs["accepted"].sum())}), flush=True)


if __name__ == "__main__":
    main()
