"""K1w (csrc/wide.hip): kernels wider than K1's register-resident halo (bw >
511, up to 32,767 -- a window of 65,535 cells, the reference's UShort
retirement count; wider kernels replay, test_ushort_*) on directional
units with a threshold > 0 -- a chunk-plane screen over each word's union
window, then every lane's FP64 score over the window's adds in ascending
position (the order the reference's deque cell receives them,
misc/peakcall.cpp:186-209), runs and peaks in K1b's record format, K2/K3
unchanged.  Every candidate region, peak, counts and FP64 peak score
bit-exact against the oracle; bin/regions tables byte-identical."""
import numpy as np
import pytest

from tests.gen import random_unit
from tests.test_cli import compare_tool, make_inputs
from tests.test_gpu_replay import compare, run_units

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bw", [512, 600, 1000, 2500, 6000])
def test_wide_single_sample(gpu_lib, oracle, bw):
    rng = np.random.default_rng(bw + 1)
    length, bg = 400_000, 0.002
    pos, cnt = random_unit(rng, length, bw, n_clusters=40)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)])
    assert len(ref) > 0
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("thr", [10.0, 25.0, 80.0])
def test_wide_thresholds_dense(gpu_lib, oracle, thr):
    """dense background (runs merge across kernels) and high stacks (escapes)"""
    rng = np.random.default_rng(int(thr))
    length, bw, bg = 300_000, 900, 0.004
    pos, cnt = random_unit(rng, length, bw, n_bg=length // 60, n_clusters=30, cluster_tags=(50, 400), sd=300)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=thr, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], region_thr=thr)
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("coeffs", [None, [0.6, 1.7]])
def test_wide_pooled_control(gpu_lib, oracle, coeffs):
    rng = np.random.default_rng(61)
    length, bw, bg, S = 250_000, 700, 0.004, 3
    pos, cnt = random_unit(rng, length, bw, S=S)
    control = [0, 1, 0]
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, control=control, coeffs=coeffs, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], control=control, coeffs=coeffs)
    compare(ref, ref_sums, regs, gcnt)


def test_wide_head_hits_and_contig_end(gpu_lib, oracle):
    """tags inside the first bw positions (quirk Q1: the K0 replay of the
    unit's start) and near the contig end (scores up to len + bw)"""
    rng = np.random.default_rng(62)
    length, bw, bg = 60_000, 1200, 0.003
    pos, cnt = random_unit(rng, length, bw, lo=1, hi=length)
    extra = {3: 5, 40: 9, 700: 30, length - 5: 40, length: 12}
    d = {int(p): int(c) for p, c in zip(pos, cnt[:, 0])}
    for p, c in extra.items():
        d[p] = d.get(p, 0) + c
    pos = np.array(sorted(d), np.uint32)
    cnt = np.array([[d[int(p)]] for p in pos], np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)])
    compare(ref, ref_sums, regs, gcnt)


def test_wide_pipelined_passes(gpu_lib, oracle):
    """K1w passes pipeline like K1's (up_run_async)"""
    capi = gpu_lib
    rng = np.random.default_rng(63)
    length, bw, bg = 200_000, 800, 0.003
    pos, cnt = random_unit(rng, length, bw)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, cap=1 << 20)
    with capi.Lib(0) as g:
        g.set_params(bw, 1, bg)
        u = g.add_unit(length)
        g.scatter(u, 0, 0, pos, cnt[:, 0])
        g.run_async()
        g.run_async()
        for _ in range(2):
            n = g.run_wait()
            regs, k = g.regions(n)
            compare(ref, ref_sums, regs.copy(), k.copy())


@pytest.mark.parametrize("bw", ["700", "2000"])
def test_wide_regions_cli(orc_bin, gpu_lib, tmp_path, bw):
    contigs = [("chrA", 200_000), ("chrB", 90_000), ("chrC", 40_000)]
    ct, files = make_inputs(tmp_path, 70 + int(bw), contigs, 2, n_cl=12, sd=200)
    out = compare_tool(orc_bin, tmp_path, "regions", ["-q", "-c", ct, "-f", "-b", bw, "-k", "0"] + files)
    assert out.count("\n") > 3


@pytest.mark.parametrize("bw", [32767, 32768, 40000, 65535])
def test_ushort_retirement_wrap(gpu_lib, oracle, bw):
    """From bw 32,768 on the window (2bw + 1 cells) exceeds the reference's
    UShort retirement count (misc/peakcall.cpp:172-177): a gap of 65,536 or
    more between adds retires (gap mod 65,536) cells -- or (2bw + 1) mod
    65,536 past 2bw -- and the rest of the window stays misaligned.  K1w
    covers bw <= 32,767 only; wider kernels take the whole-buffer replay,
    which models the wrap (emulate.hip).  Clusters 75,000 - 120,000 apart
    with nothing between them; every candidate against the oracle."""
    rng = np.random.default_rng(bw)
    length, bg = 480_000, 0.002
    d = {}
    for c, n in ((20_000, 300), (95_000, 260), (215_000, 400), (290_000, 220), (400_000, 350)):
        for o in np.rint(rng.normal(0, 80, n)).astype(np.int64):
            d[int(c + o)] = d.get(int(c + o), 0) + 1
    pos = np.array(sorted(d), np.uint32)
    cnt = np.array([[d[int(p)]] for p in pos], np.uint32)
    ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt, region_thr=0.3, kurt_thr=0.0, hit_thr=1.0, cap=1 << 20)
    regs, gcnt = run_units(gpu_lib, bw, bg, [(length, pos, cnt, None)], region_thr=0.3, kurt_thr=0.0,
                           hit_thr=1.0)
    assert len(ref) > 0
    compare(ref, ref_sums, regs, gcnt)


@pytest.mark.parametrize("bw", ["32767", "32768", "40000", "65535"])
def test_ushort_wrap_regions_cli(orc_bin, gpu_lib, tmp_path, bw):
    """bin/regions -b at and past the UShort wrap: tables byte-identical to
    the oracle CLI (three contigs per buffer, both buffers)"""
    contigs = [("chrA", 200_000), ("chrB", 90_000), ("chrC", 60_000)]
    ct, files = make_inputs(tmp_path, 7 + int(bw), contigs, 1, n_cl=5, sd=300)
    out = compare_tool(orc_bin, tmp_path, "regions",
                       ["-q", "-c", ct, "-f", "-b", bw, "-k", "0", "-r", "0.2", "-t", "1"] + files)
    assert any(line and not line.startswith("#") for line in out.splitlines())
