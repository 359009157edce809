#!/usr/bin/env python3
"""K1 probe: time the scan over hg19-sized directional units with the bench's
synthetic tags and with all-zero tracks (same bytes, no hits), to separate
the HBM floor from the per-hit work.  Prints one JSON line.

usage: k1_probe.py [--contigs N] [--reps R]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from unipeak_amd import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contigs", type=int, default=25)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--bw", type=int, default=50)
    ap.add_argument("--modes", default="synthetic,nopeaks,zeros")
    args = ap.parse_args()
    lens = [int(l.split()[1]) for l in open(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
            if l.strip()][:args.contigs]
    out = {}
    for mode in args.modes.split(","):
        with capi.Lib(0) as g:
            g.set_params(args.bw, 1, 0.00365)
            for st in (0, 1):
                for ci, L in enumerate(lens):
                    u = g.add_unit(L, buffer_id=st)
                    if mode != "zeros":
                        g.synth(u, 0, 0, 1000, ci, st, nondir=False, peaks=mode == "synthetic")
            ks, walls, kb = [], [], []
            for _ in range(args.reps):
                n = g.run()
                t = g.timings()
                ks.append(t[0])
                kb.append(t[4])
                walls.append(t[3])
            byt = 1 * 2 * sum(lens)  # uint8 per bp per strand
            k1 = float(np.median(ks))
            out[mode] = {"k1_ms": round(k1, 4), "k1b_ms": round(float(np.median(kb)), 4),
                         "GBps": round(byt / k1 / 1e6, 1),
                         "wall_ms": round(float(np.median(walls)), 4), "regions": int(n)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
