"""K1b keys (DESIGN.md §4 "K1b keys"): flags and peaks decided by the exact
integer Q(x) = sum c_h (bw^2 - (x-h)^2) instead of the FP64 walk.  These
cases aim at the three places where Q alone cannot decide and the FP64
scores must: equal Q at two positions of a run (symmetric hits; peaks tied
inside a strip and across a strip edge), thresholds inside Q's undecided
band (thr equal to, or one ulp around, an FP64 score the oracle computed),
and counts too large for uint32 Q (the pass falls back to the FP64 walk).
Everything bit-exact against the oracle."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_gpu_unit import compare, run_gpu

pytestmark = pytest.mark.gpu

STRIP = 16384


def motif_unit(rng, length, bw, centres, sep, count):
    """pairs of equal hits `sep` apart around each centre (odd sep: the two
    middle positions hold the same Q), plus background"""
    pos, cnt = random_unit(rng, length, bw, n_clusters=0)
    dense = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
    for c0, s, k in zip(centres, sep, count):
        for p in (c0, c0 + s):
            dense[p] = dense.get(p, 0) + k
    pos = np.array(sorted(dense), np.uint32)
    return pos, np.array([[dense[int(p)]] for p in pos], np.uint32)


@pytest.mark.parametrize("bw", [50, 20, 90])
def test_tied_peaks_within_and_across_strips(gpu_lib, oracle, bw):
    rng = np.random.default_rng(31 + bw)
    length = 5 * STRIP
    centres, sep, count = [], [], []
    x = 2000
    while x < length - 2000:
        centres.append(x)
        sep.append(int(rng.choice([1, 3, 5, 11, 2 * (bw // 2) + 1])))
        count.append(int(rng.integers(8, 14)))
        x += int(rng.integers(700, 1500))
    for s in range(1, 5):  # pairs straddling a strip edge: the tie spans two strips
        centres.append(s * STRIP)
        sep.append(1 if s % 2 else 3)
        count.append(12)
    pos, cnt = motif_unit(rng, length, bw, centres, sep, count)
    bg = 0.003
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, kurt_thr=0.0)
    regs, gcnt, f, _, _ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert len(regs) > 20


def test_tied_peaks_nondirectional(gpu_lib, oracle):
    rng = np.random.default_rng(77)
    length, bw, bg = 3 * STRIP, 50, 0.004
    centres = list(range(1500, length - 1500, 900))
    pos, cf = motif_unit(rng, length, bw, centres, [1] * len(centres), [9] * len(centres))
    cr = np.zeros_like(cf)
    cr[::3] = cf[::3]  # the reverse strand shares a third of the hits
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cf, cr, nondir=True, kurt_thr=0.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cf, cr, nondir=True, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert len(regs) > 10


@pytest.mark.parametrize("seed", range(3))
def test_threshold_on_an_fp64_score(gpu_lib, oracle, seed):
    """region threshold equal to (and one ulp around) scores the reference
    computes: Q cannot decide those positions, the FP64 walk must"""
    rng = np.random.default_rng(500 + seed)
    length, bw, bg = 60_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    prof = oracle.profile(bw, bg, length, pos, cnt)
    cand = prof[(prof > 5.0) & (prof < 60.0)]
    assert cand.size > 100
    for thr in rng.choice(cand, 3, replace=False):
        for t in (thr, np.nextafter(thr, np.inf), np.nextafter(thr, -np.inf)):
            ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=float(t), kurt_thr=0.0)
            regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, region_thr=float(t),
                                     kurt_thr=0.0)
            compare(ref, ref_sums, regs, gcnt)
            assert len(regs) > 0


@pytest.mark.parametrize("big", [3_000, 2_000_000])
def test_large_counts(gpu_lib, oracle, big):
    """escaped counts: 3,000 keeps Q below 2^32 (keys on), 2,000,000 cannot
    (the pass runs the FP64 walk); both exact"""
    rng = np.random.default_rng(big)
    length, bw, bg = 80_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    cnt[rng.choice(cnt.shape[0], 20, replace=False), 0] = big
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, kurt_thr=0.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)


def test_keys_with_pooled_samples_nondir_corr(gpu_lib, oracle):
    """several pooled samples use the keys only when K3 runs its own KDE
    (-D with the strand correlation): K1b keys over pooled integer counts"""
    from tests.test_gpu_unit import close
    rng = np.random.default_rng(2024)
    length, bw, bg, S = 120_000, 50, 0.004, 3
    pos, cf = random_unit(rng, length, bw, S=S)
    cr = np.roll(cf, 5, axis=0)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cf, cr, nondir=True, corr_thr=0.2, control=[0, 1, 0])
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cf, cr, nondir=True, corr_thr=0.2,
                             control=[0, 1, 0], want_corr=True)
    compare(ref, ref_sums, regs, gcnt)
    assert close(ref["corr"], regs["corr"])
    assert len(regs) > 5
