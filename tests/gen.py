"""Seeded random inputs for parity tests (sparse (pos, counts) units)."""
import numpy as np


def random_unit(rng, length, bw, S=1, n_bg=None, n_clusters=None, lo=None, hi=None,
                max_bg=3, cluster_tags=(20, 200), sd=60):
    """Sparse per-position counts [n, S] on positions lo..hi (ascending)."""
    lo = 2 * bw + 2 if lo is None else lo
    hi = length - 2 * bw - 1 if hi is None else hi
    span = hi - lo + 1
    n_bg = max(1, span // 300) if n_bg is None else n_bg
    n_clusters = max(1, span // 5000) if n_clusters is None else n_clusters
    dense = {}
    for s in range(S):
        pts = rng.integers(lo, hi + 1, n_bg)
        for p in pts:
            dense.setdefault(int(p), np.zeros(S, np.uint32))[s] += rng.integers(1, max_bg + 1)
    for _ in range(n_clusters):
        c = rng.integers(lo, hi + 1)
        n = rng.integers(*cluster_tags)
        for s in range(S):
            offs = np.rint(rng.normal(0, sd, n // S + 1)).astype(np.int64)
            for o in offs:
                p = int(c + o)
                if lo <= p <= hi:
                    dense.setdefault(p, np.zeros(S, np.uint32))[s] += 1
    pos = np.array(sorted(dense), np.uint32)
    cnt = np.array([dense[int(p)] for p in pos], np.uint32).reshape(len(pos), S)
    return pos, cnt
