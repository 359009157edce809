"""The track layout (2-bit fields, escape 3 and the overflow table) and K1's
integer screen against the oracle: escaped counts (the
screen sends their chunk to the exact path) at peaks and in the background, with
counts on both sides of each boundary, thresholds from "almost everything is a region"
to "almost nothing is", every bandwidth class of the screen window (bw 1 .. 255, NH = 1 .. 4), scaled
pooling with large and negative coefficients, and device-resident input
through up_unit_pack."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_gpu_unit import compare, run_gpu, close

pytestmark = pytest.mark.gpu


def with_big_counts(rng, pos, cnt, n, lo, hi):
    """add n positions holding counts in [lo, hi) (merged into pos/cnt)"""
    dense = {int(p): c.copy() for p, c in zip(pos, cnt)}
    S = cnt.shape[1]
    for p in rng.choice(pos, size=min(n, len(pos)), replace=False):
        v = np.zeros(S, np.uint32)
        v[int(rng.integers(0, S))] = int(rng.integers(lo, hi))
        dense[int(p)] = dense[int(p)] + v
    p = np.array(sorted(dense), np.uint32)
    return p, np.array([dense[int(x)] for x in p], np.uint32).reshape(len(p), S)


@pytest.mark.parametrize("lo,hi", [(6, 10), (13, 18), (15, 16), (128, 255), (255, 256), (255, 100_000),
                                   (1 << 20, 1 << 24)])
def test_large_counts_exact(gpu_lib, oracle, lo, hi):
    rng = np.random.default_rng(lo)
    length, bw, bg = 200_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    pos, cnt = with_big_counts(rng, pos, cnt, 40, lo, hi)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    regs, gcnt, f, _, last = run_gpu(gpu_lib, bw, bg, length, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)
    assert oracle.profile(bw, bg, length, pos, cnt).tobytes() == f.tobytes()
    assert last == pos[-1]


def test_large_counts_multi_sample_controls(gpu_lib, oracle):
    rng = np.random.default_rng(77)
    length, bw, bg, S = 120_000, 30, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    pos, cnt = with_big_counts(rng, pos, cnt, 60, 200, 5000)
    control = [0, 1, 0]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, control=control)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, control=control)
    compare(ref, ref_sums, regs, gcnt)


def test_tag_total_counts_escapes(gpu_lib):
    pos = np.array([10, 11, 20, 30, 39, 40], np.uint32)
    cnt = np.array([1, 14, 254, 15, 7, 70_000], np.uint32)
    with gpu_lib.Lib(0) as g:
        g.set_params(50, 1, 0.003)
        u = g.add_unit(1000)
        g.scatter(u, 0, 0, pos, cnt)
        assert g.tag_total(u, 0, 0) == int(cnt.sum())
        # overwrite: the escape at 40 becomes a plain nibble, 11 becomes an
        # escape, 39 (the other nibble of 40's byte) is cleared
        g.scatter(u, 0, 0, np.array([11, 39, 40], np.uint32), np.array([999, 0, 3], np.uint32))
        assert g.tag_total(u, 0, 0) == 1 + 999 + 254 + 15 + 3


@pytest.mark.parametrize("thr", [0.05, 1.0, 25.0, 400.0])
@pytest.mark.parametrize("bw", [1, 15, 16, 17, 33, 64, 127, 128, 150, 191, 192, 255, 256, 300, 383, 384, 449, 511])
def test_screen_thresholds_and_bandwidths(gpu_lib, oracle, thr, bw):
    rng = np.random.default_rng(1000 * bw + int(thr * 10))
    length, bg = 70_000, 0.003
    pos, cnt = random_unit(rng, length, bw, max_bg=4)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=thr, kurt_thr=0.0, hit_thr=1.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, region_thr=thr, kurt_thr=0.0,
                             hit_thr=1.0)
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("coeffs", [[0.37, 1.91, 0.7], [-2.5, 3.0, 0.01], [900.0, 0.5, 7.0],
                                    [1e6, 1.0, 1.0]])
def test_screen_with_coefficients(gpu_lib, oracle, coeffs):
    rng = np.random.default_rng(int(abs(coeffs[0]) * 10) % 1000)
    length, bw, bg, S = 80_000, 40, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, coeffs=coeffs, kurt_thr=0.0)
    regs, gcnt, f, _, _ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, coeffs=coeffs, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert oracle.profile(bw, bg, length, pos, cnt, coeffs=coeffs).tobytes() == f.tobytes()


def test_regions_across_strip_and_block_edges(gpu_lib, oracle):
    """clusters centred on 1024-block and 16384-strip boundaries (screen halos)"""
    rng = np.random.default_rng(5)
    length, bw, bg = 100_000, 50, 0.003
    dense = {}
    for c in [1024 * k for k in range(1, 90, 3)] + [16384 * k for k in range(1, 6)]:
        for o in np.rint(rng.normal(0, 25, 60)).astype(int):
            p = c + int(o)
            if 2 * bw + 2 <= p <= length - 2 * bw - 1:
                dense[p] = dense.get(p, 0) + 1
    pos = np.array(sorted(dense), np.uint32)
    cnt = np.array([[dense[int(p)]] for p in pos], np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)
    assert len(regs) > 20


def test_pack_from_device_array(gpu_lib, oracle):
    """device-resident dense uint32 counts (a torch tensor) -> up_unit_pack"""
    import torch
    rng = np.random.default_rng(11)
    length, bw, bg = 150_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    pos, cnt = with_big_counts(rng, pos, cnt, 20, 250, 3000)
    dense = np.zeros(length, np.uint32)
    dense[pos - 1] = cnt[:, 0]
    t = torch.from_numpy(dense.view(np.int32)).to("cuda:0")
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, bg)
        u = g.add_unit(length)
        torch.cuda.synchronize()
        g.pack(u, 0, 0, t.data_ptr())
        n = g.run()
        regs, gcnt = g.regions(n)
        assert g.tag_total(u, 0, 0) == int(cnt.sum())
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)


def test_nondir_large_counts_corr(gpu_lib, oracle):
    rng = np.random.default_rng(21)
    length, bw, bg = 100_000, 50, 0.004
    pos, cf = random_unit(rng, length, bw)
    pos, cf = with_big_counts(rng, pos, cf, 30, 255, 2000)
    cr = np.roll(cf, 5, axis=0)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cf, cr, nondir=True, corr_thr=0.2)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cf, cr, nondir=True, corr_thr=0.2,
                             want_corr=True)
    compare(ref, ref_sums, regs, gcnt)
    assert close(ref["corr"], regs["corr"])


def _edge_cluster(oracle, bw, bg, length, edge, want):
    """a tag cluster shifted until the oracle's region ends at `edge`
    (want='right') or starts at edge + 1 (want='left'): a run that K2 closes
    or opens at a strip boundary"""
    base = np.array([-30, -12, -5, 0, 4, 9, 21, 33])
    for d in range(-200, 200):
        pos = np.unique(edge + d + base).astype(np.uint32)
        cnt = np.full((len(pos), 1), 3, np.uint32)
        ref, _ = oracle.run_unit(bw, bg, pos, cnt)
        if any((r["right"] == edge) if want == "right" else (r["left"] == edge + 1) for r in ref):
            return pos, cnt
    raise AssertionError("no shift puts the region edge on the strip boundary")


def test_runs_across_whole_strips_peak_merge(gpu_lib, oracle):
    """runs spanning several 16384-position strips: K3 merges the peaks of
    their per-strip parts (first maximum, ties across strips included) and runs
    closed/opened exactly at a strip boundary"""
    rng = np.random.default_rng(99)
    length, bw, bg = 200_000, 50, 0.003
    dense = {}
    # constant density over 3+ strips: equal scores everywhere inside (ties)
    for p in range(10_000, 60_000):
        dense[p] = 1
    # random density over 4 strips with the maximum in a middle strip
    for p in range(70_000, 140_000, 3):
        dense[p] = int(rng.integers(1, 4))
    for p in range(101_000, 101_040):
        dense[p] = 40
    # a run whose maximum sits in its first (partial) strip, one in its last
    for p in range(146_000, 170_000, 2):
        dense[p] = 2
    for p in range(146_100, 146_130):
        dense[p] = 30
    for p in range(175_000, 196_000, 2):
        dense[p] = 2
    for p in range(195_900, 195_930):
        dense[p] = 30
    pos = np.array(sorted(dense), np.uint32)
    cnt = np.array([[dense[int(p)]] for p in pos], np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, kurt_thr=0.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert (ref["right"] - ref["left"] >= 16384).sum() >= 3


@pytest.mark.parametrize("want", ["right", "left"])
def test_run_edge_on_strip_boundary(gpu_lib, oracle, want):
    length, bw, bg = 60_000, 50, 0.003
    pos, cnt = _edge_cluster(oracle, bw, bg, length, 16384 * 2, want)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)


def _isolated_escapes(length, where, counts):
    dense = {}
    for p, c in zip(where, counts):
        if 1 <= p <= length:
            dense[int(p)] = dense.get(int(p), 0) + int(c)
    pos = np.array(sorted(dense), np.uint32)
    return pos, np.array([[dense[int(p)]] for p in pos], np.uint32)


@pytest.mark.parametrize("bg_tags", [False, True])
def test_isolated_escapes_strip_halo_block_edges(gpu_lib, oracle, bg_tags):
    """K1a's one-track screen bounds a strip's tags by 2 x popcount of its
    bytes, which an escaped field (count >= 3, stored as 3) breaks: the
    escape bitmap (ScanParams::esc) must send every strip whose bytes or
    halos hold one down the exact path.  Lone escapes in otherwise empty
    strips -- interior, on strip and block edges, and in the halo only
    (the first / last positions of the neighbouring strip) -- on the second
    unit of the context (global strip numbers != local ones)."""
    rng = np.random.default_rng(31 + bg_tags)
    bw, bg = 50, 0.003
    lens = [40_000, 200_000]
    S = 16384
    where = [3 * S // 2, S, S + 1, 2 * S - 120, 2 * S + 100, 3 * S + 1023, 3 * S + 1024, 5 * S + 7,
             7 * S - 40, 8 * S + 30, 1024 * 100, 1024 * 150 + 1]
    counts = [3, 4, 9, 40, 300, 70_000, 5, 12, 1000, 6, 255, 256]
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, bg)
        units = [g.add_unit(L) for L in lens]
        data = []
        for u, L in zip(units, lens):
            if u == units[0]:
                pos, cnt = random_unit(rng, L, bw)
            else:
                pos, cnt = _isolated_escapes(L, where, counts)
                if bg_tags:  # sparse background tags as well (no escapes among them)
                    extra = rng.choice(np.arange(2 * bw + 2, L - 2 * bw), size=300, replace=False)
                    d = {int(p): int(c[0]) for p, c in zip(pos, cnt)}
                    for p in extra:
                        d[int(p)] = d.get(int(p), 0) + 1
                    pos = np.array(sorted(d), np.uint32)
                    cnt = np.array([[d[int(p)]] for p in pos], np.uint32)
            g.scatter(u, 0, 0, pos, cnt[:, 0])
            data.append((pos, cnt))
        n = g.run()
        regs, gcnt = g.regions(n)
        regs, gcnt = regs.copy(), gcnt.copy()
    refs = [oracle.run_unit(bw, bg, p, c) for p, c in data]
    ref = np.concatenate([r for r, _ in refs])
    ref_sums = np.concatenate([s for _, s in refs])
    compare(ref, ref_sums, regs, gcnt)
    assert int(np.count_nonzero(regs["unit"] == units[1])) >= 8


def test_escape_added_after_a_run(gpu_lib, oracle):
    """the escape bitmap follows the tracks: an escape scattered into a
    strip that was clean in an earlier pass (and one removed) changes the
    next pass's regions exactly as the oracle's"""
    bw, bg, L = 50, 0.003, 150_000
    pos0, cnt0 = _isolated_escapes(L, [20_000], [500])
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, bg)
        u = g.add_unit(L)
        g.scatter(u, 0, 0, pos0, cnt0[:, 0])
        n0 = g.run()
        r0 = g.regions(n0)[0].copy()
        # add escapes in strips that held nothing, remove the first
        g.scatter(u, 0, 0, np.array([20_000, 70_000, 16384 * 6], np.uint32),
                  np.array([0, 800, 3], np.uint32))
        n1 = g.run()
        r1, c1 = g.regions(n1)
        r1, c1 = r1.copy(), c1.copy()
    ref0, _ = oracle.run_unit(bw, bg, pos0, cnt0)
    assert np.array_equal(ref0["left"], r0["left"]) and len(r0) == 1
    pos1, cnt1 = _isolated_escapes(L, [70_000, 16384 * 6], [800, 3])
    ref1, s1 = oracle.run_unit(bw, bg, pos1, cnt1)
    compare(ref1, s1, r1, c1)
    assert 70_000 >= r1["left"][0] and len(r1) >= 1
