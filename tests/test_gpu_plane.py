"""K1a's chunk-sum plane (kernels.h, csum_units_kernel): one byte per
16 positions, escaped fields at their counts, saturated at 255.  With one
directional pooled track and bw <= 255 the screen streams the plane instead
of the 2-bit fields.  These cases aim at the saturation (a chunk of 255 or
more tags is unbounded; with a threshold high enough that the screen's
tag budget wskip reaches 255 the saturated value must not pass as a bound),
at every window width the plane serves (R = 1..16 chunks), and at planes
rebuilt when tracks change between passes -- against the oracle.  The
index policy is UP_INDEX_ALWAYS here (the plane serves the first pass
too); tests/test_gpu_index.py runs passes without it."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_gpu_unit import compare

pytestmark = pytest.mark.gpu


def dense_unit(rng, length, bw, blocks):
    pos, cnt = random_unit(rng, length, bw)
    d = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
    for start, n, c in blocks:  # n positions of c tags each
        for p in range(start, start + n):
            d[p] = d.get(p, 0) + c
    p = np.array(sorted(d), np.uint32)
    return p, np.array([[d[int(q)]] for q in p], np.uint32)


def run(capi, bw, bg, length, pos, cnt, thr):
    with capi.Lib(0) as g:
        g.set_index_policy(capi.INDEX_ALWAYS)
        g.set_params(bw, 1, bg, region_thr=thr, kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0)
        assert g.scan_density() == (64 if bw <= 255 else 256)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        n = g.run()
        regs, c = g.regions(n)
        return regs.copy(), c.copy()


BLOCKS = [
    (30_000, 16, 20),    # one chunk of 320 tags (saturated), all escapes
    (45_008, 16, 16),    # 256 tags straddling two chunks
    (60_000, 15, 17),    # exactly 255 in one chunk
    (70_000, 1, 254),    # 254 at one position, neighbours of 1 below
    (70_001, 15, 1),
    (90_000, 32, 60),    # 1,920 tags per chunk: regions at high thresholds
    (16_384 * 7 - 8, 16, 40),  # across a strip edge (the halo of both strips)
]


@pytest.mark.parametrize("thr", [25.0, 1_500.0, 6_000.0, 20_000.0])
def test_saturated_chunks_against_oracle(gpu_lib, oracle, thr):
    rng = np.random.default_rng(7)
    bw, bg, length = 50, 0.003, 150_000
    pos, cnt = dense_unit(rng, length, bw, BLOCKS)
    regs, c = run(gpu_lib, bw, bg, length, pos, cnt, thr)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=thr)
    compare(ref, ref_sums, regs, c)
    if thr <= 6_000.0:
        assert len(ref) > 0


@pytest.mark.parametrize("bw", [1, 16, 17, 31, 48, 63, 64, 100, 127, 128, 191, 200, 240, 255, 256])
def test_plane_window_widths(gpu_lib, oracle, bw):
    """R = ceil(bw / 16) = 1 .. 16 chunks (and 256: the 2-bit stream again)"""
    rng = np.random.default_rng(bw)
    bg, length = 0.003, 180_000
    pos, cnt = dense_unit(rng, length, bw, [(16_384 * 3 - 3, 6, 4), (16_384 * 5 + 16_380, 3, 9)])
    regs, c = run(gpu_lib, bw, bg, length, pos, cnt, 25.0)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    compare(ref, ref_sums, regs, c)


def test_plane_follows_scatter_between_passes(gpu_lib, oracle):
    """a pass, then counts added, raised past 255 and cleared: the next pass
    screens the rebuilt planes"""
    bw, bg, length = 50, 0.003, 200_000
    rng = np.random.default_rng(3)
    pos, cnt = dense_unit(rng, length, bw, [(50_000, 8, 3)])
    with gpu_lib.Lib(0) as g:
        g.set_index_policy(gpu_lib.INDEX_ALWAYS)
        g.set_params(bw, 1, bg)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        g.run()
        d = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
        upd = {50_000: 0, 50_001: 0, 120_000: 300, 150_007: 2, 150_008: 2, 170_000: 1}
        for p in range(80_000, 80_016):
            upd[p] = 30
        up = np.array(sorted(upd), np.uint32)
        g.scatter(u, 0, 0, up, np.array([upd[int(p)] for p in up], np.uint32))
        n = g.run()
        regs, c = g.regions(n)
        regs, c = regs.copy(), c.copy()
    d.update(upd)
    d = {p: v for p, v in d.items() if v}
    p1 = np.array(sorted(d), np.uint32)
    c1 = np.array([[d[int(p)]] for p in p1], np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, p1, c1)
    compare(ref, ref_sums, regs, c)
    assert any(r["left"] <= 120_000 <= r["right"] for r in ref)


def test_pooled_plane_follows_pooling_changes(gpu_lib, oracle):
    """several samples screen on the unit's pooled plane (weighted by the
    screen's sample weights, both strands of a nondirectional unit): it is
    rebuilt when the control set or the coefficients change between passes
    over the same tracks"""
    rng = np.random.default_rng(11)
    bw, bg, length, S = 50, 0.003, 160_000, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    settings = [dict(control=[0, 0, 1]), dict(control=[1, 0, 0]),
                dict(control=[0, 0, 1], coeffs=[2.5, 0.4]), dict(control=[0, 0, 0])]
    got = []
    with gpu_lib.Lib(0) as g:
        g.set_index_policy(gpu_lib.INDEX_ALWAYS)
        g.set_params(bw, S, bg, **settings[0])
        u = g.add_unit(length)
        for s in range(S):
            m = cnt[:, s] != 0
            g.scatter(u, 0, s, pos[m], cnt[m, s])
        for kw in settings:
            g.set_params(bw, S, bg, region_thr=25.0, kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0, **kw)
            assert g.scan_density() == 64
            n = g.run()
            regs, c = g.regions(n)
            got.append((regs.copy(), c.copy()))
    for kw, (regs, c) in zip(settings, got):
        ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, **kw)
        compare(ref, ref_sums, regs, c)
