"""Parity of the HIP path (through the C-ABI) with the oracle, one unit at a
time: every candidate region (accepted and rejected), its peak, per-sample
counts and filters bit-exact; FP64 peak score and KDE profile bit-exact;
kurtosis and strand correlation within 1e-12 relative (north star allows
1e-6)."""
import numpy as np
import pytest

from tests.gen import random_unit

pytestmark = pytest.mark.gpu

REL = 1e-12


def close(a, b, rel=REL):
    a, b = np.asarray(a, float), np.asarray(b, float)
    both_nan = np.isnan(a) & np.isnan(b)
    ok = both_nan | (a == b) | (np.abs(a - b) <= rel * np.maximum(np.abs(a), np.abs(b)))
    return bool(np.all(ok))


def run_gpu(capi, bw, bg, length, pos, cf, cr=None, *, nondir=False, control=None,
            coeffs=None, region_thr=25.0, kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0,
            want_corr=False, strand_label=0):
    S = (cf if cf is not None else cr).shape[1]
    with capi.Lib(0) as g:
        g.set_params(bw, S, bg, region_thr=region_thr, kurt_thr=kurt_thr, corr_thr=corr_thr,
                     hit_thr=hit_thr, nondir=nondir, control=control, coeffs=coeffs,
                     want_corr=want_corr)
        u = g.add_unit(length)
        tracks = [cf] if not nondir else [cf, cr]
        for st, c in enumerate(tracks):
            for s in range(S):
                m = c[:, s] != 0
                g.scatter(u, st, s, pos[m], c[m, s])
        n = g.run()
        regs, cnt = g.regions(n)
        f, r = g.profile(u, length)
        last = g.last_add(u)
    return regs, cnt, f, r, last


def compare(ref, ref_sums, regs, cnt):
    assert len(ref) == len(regs), (len(ref), len(regs))
    for k in ("left", "right", "peak", "sum", "accepted"):
        assert np.array_equal(ref[k], regs[k]), k
    assert np.array_equal(ref_sums, cnt)
    assert ref["peak_score"].tobytes() == regs["peak_score"].tobytes()
    assert close(ref["kurtosis"], regs["kurtosis"])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("bw", [50, 20, 90])
def test_directional_single_sample(gpu_lib, oracle, seed, bw):
    rng = np.random.default_rng(seed)
    length = int(rng.integers(20_000, 300_000))
    pos, cnt = random_unit(rng, length, bw)
    bg = 0.003
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
    regs, gcnt, f, r, last = run_gpu(gpu_lib, bw, bg, length, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)
    prof = oracle.profile(bw, bg, length, pos, cnt)
    assert prof.tobytes() == f.tobytes()
    assert last == pos[-1]


@pytest.mark.parametrize("seed", range(4))
def test_reverse_buffer_unit(gpu_lib, oracle, seed):
    rng = np.random.default_rng(100 + seed)
    length, bw, bg = 120_000, 50, 0.002
    pos, cnt = random_unit(rng, length, bw)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, None, cnt, buffer_forward=False)
    regs, gcnt, f, r, _ = run_gpu(gpu_lib, bw, bg, length, pos, cnt)
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("seed", range(4))
def test_multi_sample_with_control(gpu_lib, oracle, seed):
    rng = np.random.default_rng(200 + seed)
    length, bw, bg, S = 150_000, 50, 0.004, 4
    pos, cnt = random_unit(rng, length, bw, S=S)
    control = [0, 0, 1, 0]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, control=control, hit_thr=30.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, control=control, hit_thr=30.0)
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("big", [(1_400_000_000, 1_300_000_000, 1_200_000_000),
                                 (3_000_000_000, 2_000_000_000, 7)], ids=["u32", "over"])
def test_multi_sample_huge_counts(gpu_lib, oracle, big):
    """several pooled samples sum in uint32 window words (kernels.hip WinT)
    only while no position's sum can reach 2^32: 'u32' sums 3.9e9 at one
    position on that path, 'over' (5e9 possible) takes the FP64 pooling with
    zero coefficients (api.hip pool_mode); the reference's double countSum
    (peakcall.cpp:186-200) is exact in both"""
    rng = np.random.default_rng(250)
    length, bw, bg, S = 120_000, 50, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    i = pos.size // 2
    cnt[i] = big
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, hit_thr=30.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, hit_thr=30.0)
    assert (regs["peak"] == pos[i]).any()
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("seed", range(3))
def test_coefficients_q5(gpu_lib, oracle, seed):
    rng = np.random.default_rng(300 + seed)
    length, bw, bg, S = 100_000, 50, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    coeffs = [0.37, 1.91, 0.7]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, coeffs=coeffs)
    regs, gcnt, f, _, _ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, coeffs=coeffs)
    compare(ref, ref_sums, regs, gcnt)
    prof = oracle.profile(bw, bg, length, pos, cnt, coeffs=coeffs)
    assert prof.tobytes() == f.tobytes()


@pytest.mark.parametrize("S,nondir,bw", [(9, False, 50), (9, False, 100), (36, False, 50),
                                          (3, True, 50), (12, True, 90)],
                         ids=["8s1c", "8s1c_bw100", "35s_seq", "3s_nondir", "11s_nondir_bw90"])
def test_pooled_samples(gpu_lib, oracle, S, nondir, bw):
    """several pooled samples (POOL 1, uint32 window sums) and a control:
    K3's batched per-block fetch while the (strand, sample) tracks fit one
    wave load (32), the per-sample path beyond ('35s_seq'), both strands
    without the correlation ('*_nondir'), NH 2 windows"""
    rng = np.random.default_rng(500 + S + bw)
    length, bg = 160_000, 0.004
    control = [0] * (S - 1) + [1]
    pos_f, cnt_f = random_unit(rng, length, bw, S=S)
    if not nondir:
        ref, ref_sums = oracle.run_unit(bw, bg, pos_f, cnt_f, control=control, hit_thr=30.0)
        regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos_f, cnt_f, control=control, hit_thr=30.0)
    else:
        pos_r, cnt_r = random_unit(rng, length, bw, S=S)
        allp = np.union1d(pos_f, pos_r).astype(np.uint32)
        cf = np.zeros((allp.size, S), np.uint32)
        cr = np.zeros((allp.size, S), np.uint32)
        cf[np.searchsorted(allp, pos_f)] = cnt_f
        cr[np.searchsorted(allp, pos_r)] = cnt_r
        ref, ref_sums = oracle.run_unit(bw, bg, allp, cf, cr, nondir=True, control=control, hit_thr=30.0)
        regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, allp, cf, cr, nondir=True, control=control,
                                 hit_thr=30.0)
    assert len(regs) > 5
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("seed", range(4))
def test_nondirectional_with_corr(gpu_lib, oracle, seed):
    rng = np.random.default_rng(400 + seed)
    length, bw, bg = 200_000, 50, 0.005
    pos_f, cnt_f = random_unit(rng, length, bw)
    pos_r, cnt_r = random_unit(rng, length, bw)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    cf = np.zeros((allp.size, 1), np.uint32)
    cr = np.zeros((allp.size, 1), np.uint32)
    cf[np.searchsorted(allp, pos_f)] = cnt_f
    cr[np.searchsorted(allp, pos_r)] = cnt_r
    ref, ref_sums = oracle.run_unit(bw, bg, allp, cf, cr, nondir=True, corr_thr=0.3)
    regs, gcnt, f, r, _ = run_gpu(gpu_lib, bw, bg, length, allp, cf, cr, nondir=True,
                                  corr_thr=0.3, want_corr=True)
    compare(ref, ref_sums, regs, gcnt)
    assert close(ref["corr"], regs["corr"])
    prof = oracle.profile(bw, bg, length, allp, cf, cr, nondir=True)
    assert prof.tobytes() == (f + r).tobytes()


def test_empty_unit(gpu_lib, oracle):
    regs, gcnt, f, r, last = run_gpu(gpu_lib, 50, 0.003, 5000, np.zeros(0, np.uint32),
                                     np.zeros((0, 1), np.uint32))
    assert len(regs) == 0 and last == 0 and not f.any()


def test_dense_unit_overflows_inline_records(gpu_lib, oracle):
    """Alternating narrow regions: many runs per 1024-position strip."""
    length, bw, bg = 40_000, 5, 0.01
    pos = np.arange(200, 30_000, 13, dtype=np.uint32)
    cnt = np.full((pos.size, 1), 50, np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, kurt_thr=0.0, hit_thr=1.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cnt, kurt_thr=0.0, hit_thr=1.0)
    compare(ref, ref_sums, regs, gcnt)
    assert len(regs) > 1000


def test_synthetic_track_matches_oracle_spec(gpu_lib, oracle):
    """Device synthetic generator == oracle's host generator (same spec)."""
    import ctypes
    length, bw = 400_000, 50
    pos, cnt = oracle.synth_track(1000, 3, 1, False, length, bw)
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, 0.003)
        u = g.add_unit(length)
        g.synth(u, 0, 0, 1000, 3, 1, nondir=False, peaks=True)
        n = g.run()
        f, _ = g.profile(u, length)
    ref = oracle.profile(bw, 0.003, length, pos, cnt.reshape(-1, 1))
    assert ref.tobytes() == f.tobytes()


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("bw", [50, 13, 120])
def test_head_hits_replayed_q1(gpu_lib, oracle, seed, bw):
    """Quirk Q1: tags at positions <= bw misalign the reference's window; the
    library replays the state machine there and resyncs to the parallel scan."""
    rng = np.random.default_rng(900 + seed)
    length = int(rng.integers(3_000, 60_000))
    pos, cnt = random_unit(rng, length, bw, lo=1, n_clusters=int(rng.integers(1, 6)))
    head = rng.integers(1, bw + 1, int(rng.integers(1, 6)))
    dense = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
    for p in head:
        dense[int(p)] = dense.get(int(p), 0) + int(rng.integers(5, 40))
    if seed % 2:  # a cluster right at the start keeps a region open across the resync horizon
        for o in np.rint(rng.normal(bw, bw / 2, 80)).astype(int):
            if 1 <= o <= length:
                dense[int(o)] = dense.get(int(o), 0) + 1
    pos = np.array(sorted(dense), np.uint32)
    cnt = np.array([[dense[int(p)]] for p in pos], np.uint32)
    bg = 0.003
    thr = float(rng.choice([5.0, 25.0]))
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=thr, kurt_thr=0.0)
    regs, gcnt, f, r, last = run_gpu(gpu_lib, bw, bg, length, pos, cnt, region_thr=thr, kurt_thr=0.0)
    compare(ref, ref_sums, regs, gcnt)
    assert len(regs) > 0


@pytest.mark.parametrize("seed", range(4))
def test_head_hits_nondir_with_corr(gpu_lib, oracle, seed):
    rng = np.random.default_rng(950 + seed)
    length, bw, bg = 20_000, 50, 0.003
    pos, cf = random_unit(rng, length, bw, lo=1)
    cr = np.roll(cf, 3, axis=0)
    cf[:3] += 7
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cf, cr, nondir=True, corr_thr=0.1, kurt_thr=0.0)
    regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos, cf, cr, nondir=True, corr_thr=0.1,
                             kurt_thr=0.0, want_corr=True)
    compare(ref, ref_sums, regs, gcnt)
    assert close(ref["corr"], regs["corr"])


@pytest.mark.parametrize("offset,strand", [(75, 0), (-75, 1), (-300, 0), (400, 1)])
def test_synthetic_track_offset(gpu_lib, oracle, offset, strand):
    """up_unit_synth_offset == the spec's track moved by the -s offset, with
    what leaves [1, len] dropped (the wiggle reader's bounds)"""
    length, bw = 60_000, 50
    pos, cnt = oracle.synth_track(1000, 3, strand, True, length, bw)
    p = pos.astype(np.int64) + offset
    keep = (p >= 1) & (p <= length)
    pos, cnt = p[keep].astype(np.uint32), cnt[keep]
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, 0.003)
        u = g.add_unit(length)
        g.synth(u, 0, 0, 1000, 3, strand, nondir=True, peaks=True, offset=offset)
        assert g.tag_total(u, 0, 0) == int(cnt.sum())
        g.run()
        f, _ = g.profile(u, length)
    ref = oracle.profile(bw, 0.003, length, pos, cnt.reshape(-1, 1))
    assert ref.tobytes() == f.tobytes()


@pytest.mark.parametrize("peak_seed,offset,strand,sample_seed",
                         [(7, 75, 0, 1000), (7, -75, 1, 1031), (99, 0, 0, 1005), (7, -300, 1, 1002)])
def test_synthetic_track_replicate_mode(gpu_lib, oracle, peak_seed, offset, strand, sample_seed):
    """up_unit_synth_ex (replicate mode: shared centres, per-sample heights
    and jitter, peak kinds, chunked Poisson background) == the oracle's
    orc_synth_track_ex, tag totals and dense profile bit for bit"""
    length, bw = 700_000, 50  # > 10 background chunks of 2^16 positions, a ragged last one
    pos, cnt = oracle.synth_track_ex(sample_seed, 3, strand, True, length, bw, True, offset,
                                     peak_seed)
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, 0.003)
        u = g.add_unit(length)
        g.synth(u, 0, 0, sample_seed, 3, strand, nondir=True, peaks=True, offset=offset,
                peak_seed=peak_seed)
        assert g.tag_total(u, 0, 0) == int(cnt.sum())
        g.run()
        f, _ = g.profile(u, length)
    ref = oracle.profile(bw, 0.003, length, pos, cnt.reshape(-1, 1))
    assert ref.tobytes() == f.tobytes()


@pytest.mark.parametrize("seed", range(3))
def test_shift_best_is_first_maximum_of_table(gpu_lib, seed):
    """up_shift_best == strand_shift.cpp:209-217 applied to up_shift_scan's
    table: shifts ascending, `corr > bestCorr` from -1 (NaN never wins;
    regions too short for any shift give shift 0, corr -1)"""
    rng = np.random.default_rng(500 + seed)
    length, bw = 300_000, 50
    pos_f, cnt_f = random_unit(rng, length, bw)
    pos_r, cnt_r = random_unit(rng, length, bw)
    allp = np.union1d(pos_f, pos_r).astype(np.uint32)
    cf = np.zeros((allp.size, 1), np.uint32)
    cr = np.zeros((allp.size, 1), np.uint32)
    cf[np.searchsorted(allp, pos_f)] = cnt_f
    cr[np.searchsorted(allp, pos_r)] = cnt_r
    with gpu_lib.Lib(0) as g:
        g.set_params(bw, 1, 0.004, nondir=True)
        u = g.add_unit(length)
        for st, c in enumerate((cf, cr)):
            m = c[:, 0] != 0
            g.scatter(u, st, 0, allp[m], c[m, 0])
        n = g.run()
        idx = np.arange(n, dtype=np.uint64)[::-1].copy()
        for max_shift in (0, 20, 150, 300):
            tab = g.shift_scan(idx, max_shift)
            best, bc = g.shift_best(idx, max_shift)
            for k in range(n):
                b, c = 0, -1.0
                for s in range(max_shift + 1):
                    if tab[k, s] > c:
                        b, c = s, tab[k, s]
                assert best[k] == b and bc[k] == c, (k, max_shift)


@pytest.mark.parametrize("S,nondir", [(300, False), (1024, False), (260, True)])
def test_many_samples(gpu_lib, oracle, S, nondir):
    """more than 256 samples (the reference's nExpt_ is a UShort,
    misc/peakcall.hpp:49): K3 keeps the exptSums beyond 256 in an LDS row per
    wave; pooled planes, the pooled count track and K1b's batched sample
    fetch over many tracks; two controls; per-sample counts of every
    candidate against the oracle.  1,025 samples are refused loudly."""
    rng = np.random.default_rng(1000 + S)
    length, bw, bg = 40_000, 50, 0.004
    control = [0] * S
    control[7] = control[S - 2] = 1
    pos_f, cnt_f = random_unit(rng, length, bw, S=S, n_clusters=6, n_bg=40)
    hit = 10.0 * (S - 2)
    if not nondir:
        ref, ref_sums = oracle.run_unit(bw, bg, pos_f, cnt_f, control=control, hit_thr=hit)
        regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, pos_f, cnt_f, control=control, hit_thr=hit)
    else:
        pos_r, cnt_r = random_unit(rng, length, bw, S=S, n_clusters=6, n_bg=40)
        allp = np.union1d(pos_f, pos_r).astype(np.uint32)
        cf = np.zeros((allp.size, S), np.uint32)
        cr = np.zeros((allp.size, S), np.uint32)
        cf[np.searchsorted(allp, pos_f)] = cnt_f
        cr[np.searchsorted(allp, pos_r)] = cnt_r
        ref, ref_sums = oracle.run_unit(bw, bg, allp, cf, cr, nondir=True, control=control, hit_thr=hit,
                                        corr_thr=0.3)
        regs, gcnt, *_ = run_gpu(gpu_lib, bw, bg, length, allp, cf, cr, nondir=True, control=control,
                                 hit_thr=hit, corr_thr=0.3, want_corr=True)
    assert len(ref) > 0
    compare(ref, ref_sums, regs, gcnt)
    if S == 1024:
        with gpu_lib.Lib(0) as g:
            g.set_params(bw, 1025, bg)
            g.add_unit(1000)
            with pytest.raises(gpu_lib.UpError):
                g.run()
