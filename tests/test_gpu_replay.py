"""Configurations outside the flag scan:

* region threshold <= 0 -- processPosition's leap branch is live (quirk Q11:
  the leap position joins the region without setting its left end,
  misc/peakcall.cpp:76-78), so regions are not maximal runs of flags.  With
  non-negative scores every run of processed positions is a region, found in
  parallel (K1q); a negative coefficient takes the exact
  replay below, a unit that processes position 1 a short chain of it;
* kernel bandwidth > 511 -- wider than the scan's register-resident halo
  (NH <= 8 window words; round 3 stopped at 255):
  the exact state machine on the GPU over every unit (K0 replay,
  unipeak_amd/csrc/emulate.hip); windows up to 64 KiB live in LDS, wider ones
  in global scratch.

Every candidate region (accepted and rejected), peak, counts and FP64 peak
score bit-exact against the oracle; kurtosis/correlation within 1e-12."""
import numpy as np
import pytest

from tests.gen import random_unit

pytestmark = pytest.mark.gpu


def close(a, b, rel=1e-12):
    a, b = np.asarray(a, float), np.asarray(b, float)
    ok = (np.isnan(a) & np.isnan(b)) | (a == b) | (np.abs(a - b) <= rel * np.maximum(np.abs(a), np.abs(b)))
    return bool(np.all(ok))


def run_units(capi, bw, bg, units, *, nondir=False, **kw):
    """units: [(length, pos, cf, cr)] of one buffer -> records + counts"""
    S = units[0][2].shape[1]
    with capi.Lib(0) as g:
        g.set_params(bw, S, bg, nondir=nondir, **kw)
        for length, pos, cf, cr in units:
            u = g.add_unit(length)
            for st, c in enumerate([cf] if not nondir else [cf, cr]):
                for s in range(S):
                    m = c[:, s] != 0
                    if m.any():
                        g.scatter(u, st, s, pos[m], c[m, s])
        n = g.run()
        return g.regions(n)


def compare(ref, ref_sums, regs, cnt, corr=False):
    assert len(ref) == len(regs), (len(ref), len(regs))
    for k in ("left", "right", "peak", "sum", "accepted"):
        assert np.array_equal(ref[k], regs[k]), k
    assert np.array_equal(ref_sums, cnt)
    assert ref["peak_score"].tobytes() == regs["peak_score"].tobytes()
    assert close(ref["kurtosis"], regs["kurtosis"])
    if corr:
        assert close(ref["corr"], regs["corr"])


@pytest.mark.parametrize("thr", [0.0, -1.0, -1e-300])
@pytest.mark.parametrize("seed", range(3))
def test_threshold_le_zero_q11(gpu_lib, oracle, thr, seed):
    rng = np.random.default_rng(700 + seed)
    length, bw, bg = 60_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=thr)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], region_thr=thr)
    assert len(ref) > 3
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("bw", [128, 150, 256, 300, 450, 511, 512, 1000, 2500])
def test_wide_bandwidth(gpu_lib, oracle, bw):
    """up to 511 the parallel scan (NH <= 8 window words), wider the replay"""
    rng = np.random.default_rng(bw)
    length, bg = 400_000, 0.002
    pos, cnt = random_unit(rng, length, bw, n_clusters=40)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)])
    assert len(ref) > 0
    compare(ref, ref_sums, regs, gcnt)


def test_wide_bandwidth_nondirectional_corr(gpu_lib, oracle):
    rng = np.random.default_rng(77)
    length, bw, bg = 200_000, 200, 0.004
    pos_f, cnt_f = random_unit(rng, length, bw)
    pos_r, cnt_r = random_unit(rng, length, bw)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    cf = np.zeros((allp.size, 1), np.uint32)
    cr = np.zeros((allp.size, 1), np.uint32)
    cf[np.searchsorted(allp, pos_f)] = cnt_f
    cr[np.searchsorted(allp, pos_r)] = cnt_r
    ref, ref_sums = oracle.run_unit(bw, bg, allp, cf, cr, nondir=True, corr_thr=0.3)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, allp, cf, cr)], nondir=True, corr_thr=0.3,
                           want_corr=True)
    compare(ref, ref_sums, regs, gcnt, corr=True)


def test_replay_multi_sample_control_and_coeffs(gpu_lib, oracle):
    rng = np.random.default_rng(78)
    length, bw, bg, S = 150_000, 180, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    control = [0, 1, 0]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, control=control, coeffs=[0.6, 1.7])
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], control=control,
                           coeffs=[0.6, 1.7])
    compare(ref, ref_sums, regs, gcnt)


def test_replay_refuses_pipelined_and_profile(gpu_lib):
    """bw > 511 (kMaxBw) on a nondirectional unit: outside the parallel scans
    (K1 and the directional K1w), the segmented replay"""
    capi = gpu_lib
    with capi.Lib(0) as g:
        g.set_params(600, 1, 0.003, nondir=True)
        u = g.add_unit(10_000)
        g.scatter(u, 0, 0, np.array([5000], np.uint32), np.array([3], np.uint32))
        assert g.run() >= 0
        with pytest.raises(capi.UpError):
            g.run_async()  # replay configurations run blocking only
        with pytest.raises(capi.UpError):
            g.profile(u, 10_000)


# ---- threshold <= 0 through K1q (parallel) ----------------------------------

@pytest.mark.parametrize("thr", [0.0, -2.5])
def test_q11_parallel_nondirectional_corr(gpu_lib, oracle, thr):
    rng = np.random.default_rng(810)
    length, bw, bg = 120_000, 50, 0.004
    pos_f, cnt_f = random_unit(rng, length, bw)
    pos_r, cnt_r = random_unit(rng, length, bw)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    cf = np.zeros((allp.size, 1), np.uint32)
    cr = np.zeros((allp.size, 1), np.uint32)
    cf[np.searchsorted(allp, pos_f)] = cnt_f
    cr[np.searchsorted(allp, pos_r)] = cnt_r
    ref, ref_sums = oracle.run_unit(bw, bg, allp, cf, cr, nondir=True, corr_thr=0.3, region_thr=thr)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, allp, cf, cr)], nondir=True, corr_thr=0.3,
                           want_corr=True, region_thr=thr)
    assert len(ref) > 50
    compare(ref, ref_sums, regs, gcnt, corr=True)
    assert np.all(regs["close_pos"] == 0xFFFFFFFE)  # UP_CLOSE_Q11


@pytest.mark.parametrize("coeffs", [None, [0.6, 1.7], [0.0, 2.0], [-0.5, 1.5]])
def test_q11_pooled_controls_coeffs(gpu_lib, oracle, coeffs):
    """several samples + a control (control-only adds retire positions:
    they extend the runs); a negative coefficient can make scores negative
    and takes the replay"""
    rng = np.random.default_rng(811)
    length, bw, bg, S = 150_000, 30, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    control = [0, 1, 0]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, control=control, coeffs=coeffs, region_thr=0.0,
                                    kurt_thr=0.0)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], control=control, coeffs=coeffs,
                           region_thr=0.0, kurt_thr=0.0)
    assert len(ref) > 50
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("bw", [1, 7, 64, 255])
def test_q11_dense_runs_and_spills(gpu_lib, oracle, bw):
    """a long unit with many short runs per 16,384-position strip (the
    record lists spill) and every bandwidth class of the halo"""
    rng = np.random.default_rng(812 + bw)
    length, bg = 1_500_000, 0.004
    pos, cnt = random_unit(rng, length, bw, n_bg=length // (3 * (2 * bw + 1)))  # mean gap 3 windows
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=0.0, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], region_thr=0.0)
    assert len(ref) > 300
    compare(ref, ref_sums, regs, gcnt)


def test_q11_head_unit_takes_a_replay_chain(gpu_lib, oracle):
    """an add at <= bw + 1 processes position 1: the exact replay covers the
    unit's start up to its first clean leap, K1q the rest (test_gpu_q11_heads)"""
    rng = np.random.default_rng(813)
    length, bw, bg = 50_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    pos = np.concatenate([[bw + 1], pos]).astype(np.uint32)
    cnt = np.concatenate([[[4]], cnt]).astype(np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=0.0)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], region_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert regs["close_pos"][0] != 0xFFFFFFFE  # the chain's record
    assert np.all(regs["close_pos"][1:] == 0xFFFFFFFE)  # K1q's


def test_q11_blocking_only_profile_allowed(gpu_lib, oracle):
    capi = gpu_lib
    rng = np.random.default_rng(814)
    length, bw, bg = 40_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    with capi.Lib(0) as g:
        g.set_params(bw, 1, bg, region_thr=0.0)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        assert g.run() > 0
        with pytest.raises(capi.UpError):
            g.run_async()  # K1q records are finished on the host: blocking up_run only
        f, _ = g.profile(u, length)
    assert oracle.profile(bw, bg, length, pos, cnt).tobytes() == f.tobytes()


def test_threshold_zero_after_reset_reports_nothing(gpu_lib):
    """a K1q pass (-r 0) with records, then up_reset_units and a pass over no
    unit: no region (the K1q placement status of the earlier pass must not
    be reported again)"""
    rng = np.random.default_rng(720)
    length, bw, bg = 60_000, 50, 0.003
    pos, cnt = random_unit(rng, length, bw)
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, bg, region_thr=0.0)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        assert g.run() > 3
        g.reset_units()
        assert g.run() == 0
        regs, _ = g.regions(0)
        assert len(regs) == 0
