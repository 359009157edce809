"""Pooled count tracks (UnitDesc::pct, pct_kernel): with
several pooled samples and no coefficients (POOL 1) the exact kernels (K1b,
K3, K4) read one byte per position -- the pooled samples' count sum,
saturated at 255, where the samples' own tracks are summed instead -- in
place of every sample's 2-bit track.  These cases aim at the saturation
(pooled sums of 254, 255 and far above, built from escaped fields), at
control samples (not pooled), at nondirectional units (one track per
strand) and at tracks changing between passes -- against the oracle."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_gpu_replay import compare

pytestmark = pytest.mark.gpu


def stacked_unit(rng, length, bw, S, stacks):
    pos, cnt = random_unit(rng, length, bw, S=S)
    d = {int(p): c.copy() for p, c in zip(pos, cnt)}
    for p, per_sample in stacks:  # per-sample counts at one position
        d[p] = d.get(p, np.zeros(S, np.uint32)) + np.array(per_sample, np.uint32)
    p = np.array(sorted(d), np.uint32)
    return p, np.array([d[int(q)] for q in p], np.uint32).reshape(len(p), S)


def run(capi, bw, bg, length, pos, cnt, nondir=False, cr=None, **kw):
    S = cnt.shape[1]
    with capi.Lib(0) as g:
        g.set_params(bw, S, bg, nondir=nondir, **kw)
        u = g.add_unit(length)
        for st, c in enumerate([cnt] if not nondir else [cnt, cr]):
            for s in range(S):
                m = c[:, s] != 0
                if m.any():
                    g.scatter(u, st, s, pos[m], c[m, s])
        n = g.run()
        regs, k = g.regions(n)
        return regs.copy(), k.copy()


STACKS = [(30_000, [40] * 8),              # 320: saturated, escapes in every sample
          (30_001, [31, 32, 32, 32, 32, 32, 32, 32]),  # 255 exactly
          (30_002, [30, 32, 32, 32, 32, 32, 32, 32]),  # 254
          (45_000, [3, 0, 0, 0, 0, 0, 0, 250]),        # one sample's escape >= 255
          (60_000, [2, 2, 2, 2, 2, 2, 2, 2])]          # no escape, 16


@pytest.mark.parametrize("control", [None, [0, 0, 1, 0, 0, 0, 0, 0]])
@pytest.mark.parametrize("thr", [25.0, 400.0, 2_000.0])
def test_pooled_track_saturation(gpu_lib, oracle, control, thr):
    rng = np.random.default_rng(91)
    bw, bg, length, S = 50, 0.003, 90_000, 8
    pos, cnt = stacked_unit(rng, length, bw, S, STACKS)
    kw = dict(region_thr=thr)
    if control:
        kw["control"] = control
    regs, k = run(gpu_lib, bw, bg, length, pos, cnt, **kw)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, **kw)
    compare(ref, ref_sums, regs, k)
    if thr <= 400.0:
        assert len(ref) > 0


@pytest.mark.parametrize("bw", [16, 100, 300])
def test_pooled_track_nondirectional_corr(gpu_lib, oracle, bw):
    rng = np.random.default_rng(92 + bw)
    bg, length, S = 0.003, 120_000, 4
    pos_f, cf = stacked_unit(rng, length, bw, S, [(40_000, [70, 70, 70, 70])])
    pos_r, cr_ = random_unit(rng, length, bw, S=S)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    f = np.zeros((allp.size, S), np.uint32)
    r = np.zeros((allp.size, S), np.uint32)
    f[np.searchsorted(allp, pos_f)] = cf
    r[np.searchsorted(allp, pos_r)] = cr_
    regs, k = run(gpu_lib, bw, bg, length, allp, f, nondir=True, cr=r, corr_thr=0.2, want_corr=True)
    ref, ref_sums = oracle.run_unit(bw, bg, allp, f, r, nondir=True, corr_thr=0.2)
    compare(ref, ref_sums, regs, k, corr=True)


def test_pooled_track_follows_scatter(gpu_lib, oracle):
    """a pass, then one sample's counts raised past the saturation and
    another's cleared: the next pass reads the rebuilt pooled track"""
    rng = np.random.default_rng(93)
    bw, bg, length, S = 50, 0.003, 80_000, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, S, bg)
        u = g.add_unit(length)
        for s in range(S):
            m = cnt[:, s] != 0
            g.scatter(u, 0, s, pos[m], cnt[m, s])
        g.run()
        g.scatter(u, 0, 1, np.array([20_000, 20_001], np.uint32), np.array([300, 7], np.uint32))
        m = cnt[:, 2] != 0
        g.scatter(u, 0, 2, pos[m], np.zeros(int(m.sum()), np.uint32))
        n = g.run()
        regs, k = g.regions(n)
        regs, k = regs.copy(), k.copy()
    d = {int(p): c.copy() for p, c in zip(pos, cnt)}
    for p in d:
        d[p][2] = 0
    for p, v in ((20_000, 300), (20_001, 7)):
        d.setdefault(p, np.zeros(S, np.uint32))[1] = v
    p1 = np.array(sorted(q for q in d if d[q].any()), np.uint32)
    c1 = np.array([d[int(q)] for q in p1], np.uint32).reshape(len(p1), S)
    ref, ref_sums = oracle.run_unit(bw, bg, p1, c1)
    compare(ref, ref_sums, regs, k)
    assert any(r["left"] <= 20_000 <= r["right"] for r in ref)
