"""Wider draw-order search for the survey's PCG64 seed-11 probe input, on the
chr21-only table ("synthetic chr21 wig (352,614 tags)", same
spec).  Only the input tag count is matched; see tools/pcg11_search.py.
Usage: python tools/pcg11_search2.py [workers]"""
import itertools
import sys
from multiprocessing import Pool

import numpy as np

LAM, BW = 0.002925, 50
L = 48129895
WANT = 352614


def run(v):
    rng = np.random.default_rng(11)
    lo, hi = 2 * BW + 2, L - 2 * BW - 1
    total = 0

    def bg():
        if v["bg"] == "dense":
            return int(rng.poisson(LAM, hi - lo + 1).sum())
        mean = LAM * L if v["bg"] == "L" else LAM * (hi - lo + 1)
        n = int(rng.poisson(mean))
        if v["bgpos"] == "inc":
            rng.integers(lo, hi + 1, n)
        elif v["bgpos"] == "exc":
            rng.integers(lo, hi, n)
        else:
            rng.uniform(lo, hi + 1, n)
        return n

    npk = max(1, L // 150000) if v["npk"] == "floor" else max(1, round(L / 150000))
    clo, chi = 10**4, L - 10**4

    def centres():
        if v["cdraw"] == "inc":
            return rng.integers(clo, chi + 1, npk)
        if v["cdraw"] == "exc":
            return rng.integers(clo, chi, npk)
        return rng.uniform(clo, chi, npk)

    def sizes():
        return rng.integers(20, 200, npk)

    def peaks(cs, ns):
        t = 0
        if v["vec"]:
            if cs is None:
                cs = centres()
            if ns is None:
                ns = sizes()
            if v["norm"] == "flat":
                rng.normal(0, 60, int(ns.sum()))
            else:
                for c, n in zip(cs, ns):
                    rng.normal(c, 60, int(n))
            return int(ns.sum())
        for j in range(npk):
            if cs is None:
                if v["cdraw"] == "inc":
                    c = rng.integers(clo, chi + 1)
                elif v["cdraw"] == "exc":
                    c = rng.integers(clo, chi)
                else:
                    c = rng.uniform(clo, chi)
            else:
                c = cs[j]
            n = int(rng.integers(20, 200)) if ns is None else int(ns[j])
            rng.normal(c, 60, n)
            t += n
        return t

    cs = ns = None
    if v["share"] in ("c", "cn"):
        cs = centres()
        if v["share"] == "cn":
            ns = sizes()
    if v["group"] == "strand":
        for _ in range(2):
            if v["bgfirst"]:
                total += bg() + peaks(cs, ns)
            else:
                total += peaks(cs, ns) + bg()
    elif v["group"] == "bgall":
        total += bg() + bg() + peaks(cs, ns) + peaks(cs, ns)
    else:
        total += peaks(cs, ns) + peaks(cs, ns) + bg() + bg()
    return total, v


def variants():
    dims = dict(bg=["L", "range", "dense"], bgpos=["inc", "exc", "unif"], bgfirst=[True, False],
                group=["strand", "bgall", "pkall"], share=["none", "c", "cn"],
                cdraw=["inc", "exc", "unif"], vec=[True, False], norm=["each", "flat"],
                npk=["floor", "round"])
    names = list(dims)
    seen = set()
    for combo in itertools.product(*(dims[k] for k in names)):
        v = dict(zip(names, combo))
        if v["bg"] == "dense":
            v["bgpos"] = "-"
        if v["group"] != "strand":
            v["bgfirst"] = "-"
        if not v["vec"]:
            v["norm"] = "-"
        k = tuple(sorted(v.items()))
        if k in seen:
            continue
        seen.add(k)
        yield v


if __name__ == "__main__":
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    vs = list(variants())
    print(len(vs), "variants", flush=True)
    with Pool(w) as p:
        for t, v in p.imap_unordered(run, vs, chunksize=4):
            if t == WANT or abs(t - WANT) < 3:
                print(("MATCH " if t == WANT else "near  ") + f"{t} {v}", flush=True)
    print("done", flush=True)
