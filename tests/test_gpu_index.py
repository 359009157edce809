"""The index policy (include/unipeak_hip.h up_set_index_policy; DESIGN.md §3
"Index policy").  A pass without the per-dataset index (chunk-sum planes,
pooled planes, pooled count tracks) reads only the packed tracks: K1a
streams the 2-bit fields (kModeScreenF), K1b/K3/K4 pool the samples' own
tracks, K3's exptSums read dwords instead of plane bytes.  Every case runs
under NEVER, AUTO (first pass without, then built, then with) and ALWAYS,
pipelined and blocking, and every pass must give the oracle's records
bit for bit -- the reference makes one pass per run (src/regions.cpp:311-391)
and the index may only ever save work."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_gpu_unit import close, compare

pytestmark = pytest.mark.gpu

CASES = {
    # name: S, nondir, bw, control, coeffs, corr
    "dir1_bw50": (1, False, 50, None, None, False),
    "dir1_bw200": (1, False, 200, None, None, False),
    "dir1_bw400": (1, False, 400, None, None, False),
    "4s1c_pct": (4, False, 50, [0, 0, 1, 0], None, False),
    "9s1c_pct_bw100": (9, False, 100, [0] * 8 + [1], None, False),
    "3s_coeffs": (3, False, 50, None, [0.37, 1.91, 0.7], False),
    "nondir1_corr": (1, True, 50, None, None, True),
    "nondir3_corr": (3, True, 90, [0, 1, 0], None, True),
}


def make_case(name, seed=0):
    S, nondir, bw, control, coeffs, corr = CASES[name]
    rng = np.random.default_rng(900 + seed + 17 * len(name))
    length, bg = 180_000, 0.004
    pos_f, cnt_f = random_unit(rng, length, bw, S=S)
    # a few escaped counts (>= 3) and a saturated chunk (>= 255 tags)
    d = {int(p): c.copy() for p, c in zip(pos_f, cnt_f)}
    for p, c in ((40_000, 7), (40_001, 300), (90_000, 3)):
        d.setdefault(p, np.zeros(S, np.uint32))[0] += c
    pos_f = np.array(sorted(d), np.uint32)
    cnt_f = np.array([d[int(p)] for p in pos_f], np.uint32).reshape(-1, S)
    if not nondir:
        return dict(S=S, nondir=False, bw=bw, control=control, coeffs=coeffs, corr=corr, length=length,
                    bg=bg, pos=pos_f, cf=cnt_f, cr=None)
    pos_r, cnt_r = random_unit(rng, length, bw, S=S)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    cf = np.zeros((allp.size, S), np.uint32)
    cr = np.zeros((allp.size, S), np.uint32)
    cf[np.searchsorted(allp, pos_f)] = cnt_f
    cr[np.searchsorted(allp, pos_r)] = cnt_r
    return dict(S=S, nondir=True, bw=bw, control=control, coeffs=coeffs, corr=corr, length=length, bg=bg,
                pos=allp, cf=cf, cr=cr)


def oracle_of(oracle, c):
    hit = 10.0 * (c["S"] - sum(c["control"] or []))
    return oracle.run_unit(c["bw"], c["bg"], c["pos"], c["cf"], c["cr"], nondir=c["nondir"],
                           control=c["control"], coeffs=c["coeffs"], hit_thr=hit,
                           corr_thr=0.3 if c["corr"] else -1.0)


def open_ctx(capi, c, policy):
    g = capi.Lib(0)
    g.set_index_policy(policy)
    hit = 10.0 * (c["S"] - sum(c["control"] or []))
    g.set_params(c["bw"], c["S"], c["bg"], region_thr=25.0, kurt_thr=50.0, hit_thr=hit,
                 corr_thr=0.3 if c["corr"] else -1.0, nondir=c["nondir"], control=c["control"],
                 coeffs=c["coeffs"], want_corr=c["corr"])
    u = g.add_unit(c["length"])
    tracks = [c["cf"]] if not c["nondir"] else [c["cf"], c["cr"]]
    for st, t in enumerate(tracks):
        for s in range(c["S"]):
            m = t[:, s] != 0
            g.scatter(u, st, s, c["pos"][m], t[m, s])
    return g


def check(ref, ref_sums, regs, cnt, corr):
    compare(ref, ref_sums, regs, cnt)
    if corr:
        assert close(ref["corr"], regs["corr"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_policies_blocking(gpu_lib, oracle, name):
    c = make_case(name)
    ref, ref_sums = oracle_of(oracle, c)
    assert len(ref) > 3
    for policy, expect in ((gpu_lib.INDEX_NEVER, [(False, 0)] * 3),
                           (gpu_lib.INDEX_AUTO, [(False, 0), (True, 1), (True, 1)]),
                           (gpu_lib.INDEX_ALWAYS, [(True, 1)] * 3)):
        g = open_ctx(gpu_lib, c, policy)
        try:
            for k in range(3):
                n = g.run()
                regs, cnt = g.regions(n)
                check(ref, ref_sums, regs, cnt, c["corr"])
                assert g.index_state() == expect[k], (policy, k, g.index_state())
        finally:
            g.close()


@pytest.mark.parametrize("name", ["dir1_bw50", "9s1c_pct_bw100", "nondir3_corr"])
def test_auto_transition_while_pipelined(gpu_lib, oracle, name):
    """AUTO builds the index at the second up_run_async while the first pass
    (without it) is in flight: both passes' records stay the oracle's"""
    c = make_case(name, seed=1)
    ref, ref_sums = oracle_of(oracle, c)
    g = open_ctx(gpu_lib, c, gpu_lib.INDEX_AUTO)
    try:
        for _ in range(4):
            g.run_async()
        for _ in range(4):
            n = g.run_wait()
            regs, cnt = g.regions(n)
            check(ref, ref_sums, regs, cnt, c["corr"])
        assert g.index_state() == (True, 1)
    finally:
        g.close()


def test_invalidate_and_track_changes(gpu_lib, oracle):
    """up_invalidate_index and a scatter between passes make AUTO run the next
    pass without the index again and rebuild it for the one after"""
    c = make_case("4s1c_pct", seed=2)
    g = open_ctx(gpu_lib, c, gpu_lib.INDEX_AUTO)
    try:
        ref, ref_sums = oracle_of(oracle, c)
        for _ in range(2):
            regs, cnt = g.regions(g.run())
            check(ref, ref_sums, regs, cnt, False)
        assert g.index_state() == (True, 1)
        g.invalidate_index()
        regs, cnt = g.regions(g.run())
        check(ref, ref_sums, regs, cnt, False)
        assert g.index_state() == (False, 1)
        regs, cnt = g.regions(g.run())
        check(ref, ref_sums, regs, cnt, False)
        assert g.index_state() == (True, 2)
        # counts change: a new peak in sample 1
        add = np.arange(120_000, 120_040, dtype=np.uint32)
        g.scatter(0, 0, 1, add, np.full(add.size, 9, np.uint32))
        d = {int(p): r.copy() for p, r in zip(c["pos"], c["cf"])}
        for p in add:
            d.setdefault(int(p), np.zeros(c["S"], np.uint32))[1] = 9
        c["pos"] = np.array(sorted(d), np.uint32)
        c["cf"] = np.array([d[int(p)] for p in c["pos"]], np.uint32).reshape(-1, c["S"])
        ref, ref_sums = oracle_of(oracle, c)
        assert any(r["left"] <= 120_000 <= r["right"] for r in ref)
        for k in range(2):
            regs, cnt = g.regions(g.run())
            check(ref, ref_sums, regs, cnt, False)
            assert g.index_state() == ((False, 2) if k == 0 else (True, 3))
    finally:
        g.close()


@pytest.mark.parametrize("bw2", [300, 700, 2000])
def test_unit_regrows_for_a_wider_kernel(gpu_lib, oracle, bw2):
    """units added at -b 50 are padded for kernels up to 511; a later wider
    -b regrows them (tracks copied to the new stride) -- the windows past the
    contig end (quirk Q16) must still read zeros"""
    rng = np.random.default_rng(77 + bw2)
    length, bg = 60_000, 0.004
    pos, cnt = random_unit(rng, length, 50, lo=200, hi=length)
    with gpu_lib.Lib(0) as g:
        g.set_params(50, 1, bg)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        g.run()
        g.set_params(bw2, 1, bg, region_thr=25.0, kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0)
        regs, c = g.regions(g.run())
        regs, c = regs.copy(), c.copy()
    ref, ref_sums = oracle.run_unit(bw2, bg, pos, cnt)
    assert len(ref) > 0
    compare(ref, ref_sums, regs, c)
