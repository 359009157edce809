#!/usr/bin/env python3
"""Write the bench's synthetic samples (SURVEY.md 8(d) generator, restated
in oracle/orc_synth.c) as wiggle files, for end-to-end CLI timing of
bin/regions against the oracle CLI on identical inputs.

usage: python -m tests.make_wig OUTDIR [--table hg19|chr21] [--samples S]
       [--nondir] [--controls C]

Sample i uses seed 1000+i; controls (background only) 2000+j.  Writes
OUTDIR/contigs.txt and OUTDIR/s<i>.wig / c<j>.wig."""
import argparse
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def contig_table(name):
    rows = [l.split() for l in open(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
            if l.strip() and not l.startswith("#")]
    rows = [(r[0], int(r[1])) for r in rows]
    if name == "chr21":
        rows = [r for r in rows if r[0] == "chr21"]
    return rows


def write_sample(path, name, orc, contigs, seed, nondir, peaks, bw=50, index=None,
                 workers=8):
    """One directional wig (both strand tracks) of the synthetic spec.
    contigs: [(name, length)]; index: the generator's contig index of each
    (default 0..n-1, i.e. the position in the table the generator keys on)."""
    index = list(range(len(contigs))) if index is None else index
    with ThreadPoolExecutor(workers) as ex:
        def one(st, ci, L):
            pos, cnt = orc.synth_track(seed, ci, st, nondir, L, bw, peaks)
            return int(cnt.sum(dtype=np.uint64)), orc.format_pairs(pos, cnt, st == 1)
        jobs = {(st, k): ex.submit(one, st, index[k], L)
                for st in (0, 1) for k, (_, L) in enumerate(contigs)}
        total = sum(f.result()[0] for f in jobs.values())
        with open(path, "wb") as f:
            f.write(f"# original_file=synthetic seed {seed}\n# tags={total}\n".encode())
            for st in (0, 1):
                if st == 0:
                    f.write(f'track name="{name} +" description="{name}" priority=3 '
                            'visibility=full type=wiggle_0 alwaysZero=on color=0,0,255\n'.encode())
                else:
                    f.write(f'track name="{name} -" description=" " priority=3 visibility=full '
                            'type=wiggle_0 alwaysZero=on color=255,0,0 altColor=255,0,0\n'.encode())
                for k, (c, _) in enumerate(contigs):
                    t = jobs[(st, k)].result()[1]
                    if t:
                        f.write(f"variableStep chrom={c}\n".encode())
                        f.write(t)
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--table", default="hg19", choices=["hg19", "chr21"])
    ap.add_argument("--samples", type=int, default=1)
    ap.add_argument("--controls", type=int, default=0)
    ap.add_argument("--nondir", action="store_true")
    a = ap.parse_args()
    from tests.oracle_binding import Oracle
    from tests.conftest import _ensure_oracle
    _ensure_oracle()
    orc = Oracle()
    os.makedirs(a.outdir, exist_ok=True)
    contigs = contig_table(a.table)
    with open(os.path.join(a.outdir, "contigs.txt"), "w") as f:
        for c, L in contigs:
            f.write(f"{c}\t{L}\n")
    for i in range(a.samples):
        n = write_sample(os.path.join(a.outdir, f"s{i}.wig"), f"s{i}", orc, contigs, 1000 + i,
                         a.nondir, True)
        print(f"s{i}: {n} tags", file=sys.stderr)
    for j in range(a.controls):
        n = write_sample(os.path.join(a.outdir, f"c{j}.wig"), f"c{j}", orc, contigs, 2000 + j,
                         a.nondir, False)
        print(f"c{j}: {n} tags", file=sys.stderr)


if __name__ == "__main__":
    main()
