"""The oracle's in-process genome driver (orc_genome_unit) and the
replicate-mode generator (orc_synth_track_ex), on the CPU: the driver that
checks configs[4] at full size must give exactly what the matrix path
(orc_run_unit over host count matrices, used by every other genome test)
gives on the same units."""
import numpy as np
import pytest

from tests.test_gpu_genome import load_tables, oracle_genome_unit, oracle_unit

BW = 50


def _same(a, b):
    (ra, sa), (rb, sb) = a, b
    assert len(ra) == len(rb) > 0
    assert ra.tobytes() == rb.tobytes()  # coordinates, sums, scores, kurtosis, corr: every bit
    assert np.array_equal(sa, sb)


@pytest.mark.parametrize("S,n_ctl,nondir,buf", [(1, 0, False, 0), (1, 0, False, 1), (3, 1, False, 0),
                                                (4, 0, True, 0)])
def test_genome_unit_equals_matrix_path(oracle, S, n_ctl, nondir, buf):
    contigs = load_tables(["hg19"])
    ci = [n for n, _ in contigs].index("chrM") if S == 1 else 24
    ci = [n for n, _ in contigs].index("chr21") if nondir else ci
    contigs = [(n, min(L, 6_000_000)) for n, L in contigs]  # a 6 Mbp slice keeps it quick
    corr = 0.2 if nondir else -1.0
    thr = 5.0 if S > 1 else 25.0
    a = oracle_unit(oracle, contigs, (ci, buf), S, n_ctl, nondir, 50.0, corr, 0.004, region_thr=thr)
    b = oracle_genome_unit(oracle, contigs, (ci, buf), S, n_ctl, nondir, 50.0, corr, 0.004,
                           region_thr=thr)
    _same(a, b)


def test_synth_ex_without_peak_seed_is_the_shifted_spec(oracle):
    L = 300_000
    p0, c0 = oracle.synth_track(1000, 3, 1, True, L, BW)
    for off in (0, 75, -75, -300):
        p, c = oracle.synth_track_ex(1000, 3, 1, True, L, BW, True, off, 0)
        q = p0.astype(np.int64) + off
        keep = (q >= 1) & (q <= L)
        assert np.array_equal(p, q[keep]) and np.array_equal(c, c0[keep])


def test_replicates_share_peak_centres(oracle):
    """replicate mode: two samples' peaks sit within the jitter of each other;
    the survey spec's samples have unrelated peaks"""
    L = 3_000_000

    def peak_sites(seed, peak_seed):
        p, c = oracle.synth_track_ex(seed, 5, 0, True, L, BW, True, 0, peak_seed)
        return set((p[c >= 2] // 1000).tolist())  # 1 kb bins holding stacked tags

    a, b = peak_sites(1000, 7), peak_sites(1001, 7)
    assert len(a & b) > 0.6 * min(len(a), len(b))
    a, b = peak_sites(1000, 0), peak_sites(1001, 0)
    assert len(a & b) < 0.2 * min(len(a), len(b))


def test_replicate_unit_filters_decide(oracle):
    """configs[4]'s replicate workload on one contig: pooled peaks cross
    -r 25 and both the correlation and the kurtosis filter reject some"""
    contigs = load_tables(["hg19", "mm9"])
    ci = [n for n, _ in contigs].index("hg19_chr22")
    contigs = [(n, min(L, 12_000_000)) for n, L in contigs]
    bg = 0.002925 * 2 * 32 * 5_750_605_500 / (5_750_605_500 & 0xFFFFFFFF)
    r, _ = oracle_genome_unit(oracle, contigs, (ci, 0), 32, 0, True, 50.0, 0.3, bg,
                              peak_seed=7, shift=75)
    assert len(r) > 40
    rej = r[r["accepted"] == 0]
    assert np.any(rej["corr"] < 0.3) and np.any(rej["kurtosis"] > 50.0)
