"""Search for the draw order of the survey's hg19 probe input.

The survey recorded, for "numpy PCG64, seed 11, one sample", only the input
fingerprint -- 22,630,558 tags / 21,483,487 nonzero (strand, position) entries
on hg19, 352,614 tags on chr21 -- and the reference's answer on it (41,113
regions + 330 rejected).  This script enumerates plausible draw orders of the
survey's spec and reports which reproduce the INPUT fingerprint; the answer is
never used to choose.  Usage: python tools/pcg11_search.py [chr21|hg19]
"""
import itertools
import sys

import numpy as np

LAM = 0.002925
BW = 50


def contigs(which):
    rows = []
    with open("unipeak_amd/data/hg19.txt") as fh:
        for line in fh:
            n, l = line.split()
            rows.append((n, int(l)))
    if which == "chr21":
        rows = [r for r in rows if r[0] == "chr21"]
    return rows


def gen(rows, v, seed=11):
    rng = np.random.default_rng(seed)
    total = 0
    nnz = 0
    c21 = 0

    def bg(L):
        lo, hi = 2 * BW + 2, L - 2 * BW - 1
        mean = LAM * L if v["bgmean"] == "L" else LAM * (hi - lo + 1)
        n = rng.poisson(mean)
        if v["bgpos"] == "int_ep":
            return rng.integers(lo, hi, n, endpoint=True)
        if v["bgpos"] == "int_ex":
            return rng.integers(lo, hi + 1, n)
        if v["bgpos"] == "int_hi":
            return rng.integers(lo, hi, n)
        if v["bgpos"] == "unif":
            return np.floor(rng.uniform(lo, hi + 1, n)).astype(np.int64)
        raise KeyError

    def centres(L):
        npk = npeaks(L)
        clo, chi = crange(L)
        if v["cend"]:
            return rng.integers(clo, chi, npk, endpoint=True)
        return rng.integers(clo, chi, npk)

    def npeaks(L):
        if v["npk"] == "floor":
            return max(1, L // 150000)
        return max(1, int(round(L / 150000)))

    def crange(L):
        if L > 2 * 10**4 + 1000:
            return 10**4, L - 10**4
        return 2 * BW + 200, L - 2 * BW - 200

    def shared_peaks(cs, ns):
        if ns is None:
            ns = rng.integers(20, 200, len(cs))
        out = []
        if v["norm"] == "each":
            for c, n in zip(cs, ns):
                out.append(np.round(rng.normal(c, 60, n)))
        else:
            offs = rng.normal(0, 60, int(ns.sum()))
            out.append(np.round(np.repeat(cs, ns) + offs))
        return np.concatenate(out).astype(np.int64)

    def peaks(L):
        if v["npk"] == "floor":
            npk = max(1, L // 150000)
        elif v["npk"] == "round":
            npk = max(1, int(round(L / 150000)))
        else:
            npk = max(1, int(np.ceil(L / 150000)))
        if L > 2 * 10**4 + 1000:
            clo, chi = 10**4, L - 10**4
        else:
            clo, chi = 2 * BW + 200, L - 2 * BW - 200
        out = []
        if v["pk"] == "vec":
            if v["cend"]:
                cs = rng.integers(clo, chi, npk, endpoint=True)
            else:
                cs = rng.integers(clo, chi, npk)
            ns = rng.integers(20, 200, npk)
            if v["norm"] == "each":
                for c, n in zip(cs, ns):
                    out.append(np.round(rng.normal(c, 60, n)))
            else:
                offs = rng.normal(0, 60, int(ns.sum()))
                out.append(np.round(np.repeat(cs, ns) + offs))
        else:
            for _ in range(npk):
                if v["cend"]:
                    c = rng.integers(clo, chi, endpoint=True)
                else:
                    c = rng.integers(clo, chi)
                n = rng.integers(20, 200)
                out.append(np.round(rng.normal(c, 60, n)))
        return np.concatenate(out).astype(np.int64)

    tracks = []
    if v["loop"] == "cs":
        order = [(ci, s) for ci in range(len(rows)) for s in (0, 1)]
    else:
        order = [(ci, s) for s in (0, 1) for ci in range(len(rows))]
    share = v.get("share", "none")
    for ci, s in order:
        L = rows[ci][1]
        if share != "none":
            if s == 0:
                cs = centres(L)
                ns = rng.integers(20, 200, len(cs)) if share == "cn" else None
            if v["bgfirst"]:
                a = bg(L)
                b = shared_peaks(cs, ns)
            else:
                b = shared_peaks(cs, ns)
                a = bg(L)
        elif v["bgfirst"]:
            a = bg(L)
            b = peaks(L)
        else:
            b = peaks(L)
            a = bg(L)
        p = np.concatenate([a, b])
        p = p[(p >= 1) & (p <= L)]
        total += p.size
        nnz += np.unique(p).size
        if rows[ci][0] == "chr21":
            c21 += p.size
    return total, nnz, c21


def variants():
    keys = dict(loop=["cs", "sc"], bgfirst=[True, False], bgmean=["L", "range"],
                bgpos=["int_ep", "int_hi", "unif"], npk=["floor", "round"],
                pk=["vec", "loop"], cend=[False, True], norm=["each", "flat"])
    names = list(keys)
    for combo in itertools.product(*(keys[k] for k in names)):
        v = dict(zip(names, combo))
        if v["pk"] == "loop" and v["norm"] == "flat":
            continue
        yield v
        if v["pk"] == "vec" and v["loop"] == "cs":
            for sh in ("c", "cn"):
                yield dict(v, share=sh)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "chr21"
    rows = contigs(which)
    want = {"chr21": (352614, None), "hg19": (22630558, 21483487)}[which]
    seen = set()
    for v in variants():
        if which == "chr21":
            v["loop"] = "cs"
        key = tuple(sorted(v.items()))
        if key in seen:
            continue
        seen.add(key)
        t, z, c21 = gen(rows, v)
        hit = t == want[0] and (want[1] is None or z == want[1])
        hit21 = c21 == 352614
        print(("MATCH " if hit else "      ") + ("C21 " if hit21 else "    ")
              + f"{t:>10} {z:>10} {c21:>8} {v}", flush=True)
