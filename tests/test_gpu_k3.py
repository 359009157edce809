"""K3 for one directional sample (csrc/stats1.hip): batched ordered sums.

The batched kernel lists every region's hit positions and runs the
sequential FP64 sums (kurtosis, peak score) one region per lane.  These
cases aim at its bookkeeping -- batches of 64 regions, pair lists that fill
mid-region (sums carried over chunks), regions too long to stage (> 4,032
positions), tied Q keys (the region's own KDE), peaks whose run crossed a
strip edge -- and compare it with the oracle and, bit for bit, with the
general K3 (UNIPEAK_K3_ONE=0)."""
import os

import numpy as np
import pytest

from tests.gen import random_unit

pytestmark = pytest.mark.gpu

FIELDS = ("unit", "left", "right", "peak", "sum", "nonctl_sum", "accepted", "close_pos")


def wide_unit(rng, length, bw):
    """background + ordinary clusters + a few dense wide blocks (hundreds to
    thousands of hit positions per region) and blocks across strip edges"""
    pos, cnt = random_unit(rng, length, bw, n_clusters=length // 3000)
    dense = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
    starts = list(rng.integers(10_000, length - 20_000, 6)) + [16_384 - 700, 3 * 16_384 - 2_000]
    for k, a in enumerate(starts):
        n = [600, 1_500, 3_000, 4_500, 9_000, 800, 1_400, 4_000][k]
        for p in range(int(a), int(a) + n):
            if rng.random() < 0.7:
                dense[p] = dense.get(p, 0) + int(rng.integers(1, 5))
    p = np.array(sorted(dense), np.uint32)
    return p, np.array([[dense[int(q)]] for q in p], np.uint32)


def run(capi, bw, bg, length, pos, cnt, one, kurt_thr=50.0):
    old = os.environ.get("UNIPEAK_K3_ONE")
    os.environ["UNIPEAK_K3_ONE"] = "1" if one else "0"
    try:
        with capi.Lib(0) as g:
            g.set_params(bw, 1, bg, region_thr=25.0, kurt_thr=kurt_thr, corr_thr=-1.0, hit_thr=10.0)
            u = g.add_unit(length)
            g.scatter(u, 0, 0, pos, cnt[:, 0])
            n = g.run()
            return g.regions(n)
    finally:
        if old is None:
            del os.environ["UNIPEAK_K3_ONE"]
        else:
            os.environ["UNIPEAK_K3_ONE"] = old


def same_bits(a, b):
    assert len(a) == len(b)
    for k in FIELDS:
        assert np.array_equal(a[k], b[k]), k
    for k in ("peak_score", "kurtosis", "corr"):
        assert a[k].tobytes() == b[k].tobytes(), k


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("bw", [50, 20, 120])
def test_batched_k3_matches_oracle_and_general_k3(gpu_lib, oracle, seed, bw):
    rng = np.random.default_rng(100 + seed)
    length = 400_000
    pos, cnt = wide_unit(rng, length, bw)
    bg = 0.003
    regs1, c1 = run(gpu_lib, bw, bg, length, pos, cnt, one=True)
    regs0, c0 = run(gpu_lib, bw, bg, length, pos, cnt, one=False)
    same_bits(regs1, regs0)
    assert np.array_equal(c1, c0)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    assert len(ref) == len(regs1) > 64  # more than one batch
    for k in ("left", "right", "peak", "sum", "accepted"):
        assert np.array_equal(ref[k], regs1[k]), k
    assert np.array_equal(ref_sums, c1)
    assert ref["peak_score"].tobytes() == regs1["peak_score"].tobytes()
    a, b = ref["kurtosis"], regs1["kurtosis"]
    assert np.all((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b)))
    spans = regs1["right"].astype(np.int64) - regs1["left"] + 1
    assert spans.max() > 4_032  # a region too long to stage
    assert (spans > 448).sum() >= 3  # regions whose pairs fill a list


def test_batched_k3_tied_keys(gpu_lib, oracle):
    """two positions holding the run's largest Q: the first maximum of the
    FP64 scores decides (the region's KDE inside the batched kernel)"""
    bw, bg, length = 50, 0.003, 60_000
    dense = {}
    # equal counts at c and c + 1 (and a symmetric flank): Q(c) == Q(c + 1) is
    # the run's largest key, at two positions
    for c in (10_000, 20_000, 30_000, 16_384 * 2 - 1):
        for d, n in ((0, 10), (1, 10), (-30, 3), (31, 3)):
            dense[c + d] = dense.get(c + d, 0) + n
    pos = np.array(sorted(dense), np.uint32)
    cnt = np.array([[dense[int(p)]] for p in pos], np.uint32)
    regs1, c1 = run(gpu_lib, bw, bg, length, pos, cnt, one=True)
    regs0, c0 = run(gpu_lib, bw, bg, length, pos, cnt, one=False)
    same_bits(regs1, regs0)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    for k in ("left", "right", "peak", "sum", "accepted"):
        assert np.array_equal(ref[k], regs1[k]), k
    assert ref["peak_score"].tobytes() == regs1["peak_score"].tobytes()
