"""Drop-in parity of the C++ CLIs (bin/) with the oracle's restatement of the
reference CLIs: byte-identical region tables, strand_shift reports and
tags_in_regions tables on seeded synthetic wiggle inputs.

Every CLI needs the GPU (gpu marker); bin/tags_in_regions is tested in
tests/test_gpu_tir.py."""
import os
import zlib
import subprocess

import numpy as np
import pytest

from tests.wig import write_contigs, write_wig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def gen_sample(rng, contigs, lo=300, n_bg=None, n_cl=None, shift_rev=0, sd=60):
    """{contig: [(pos, count)]} for both strands, positions >= lo; reverse
    clusters sit shift_rev downstream of the forward ones (fragment ends)."""
    fwd, rev = {}, {}
    for name, L in contigs:
        hi = L - 300
        nc = max(1, (hi - lo) // 6000) if n_cl is None else n_cl
        centres = [int(c) for c in rng.integers(lo + 200, hi - 200, nc)]
        for strand, d in ((0, fwd), (1, rev)):
            dense = {}
            nb = max(1, (hi - lo) // 400) if n_bg is None else n_bg
            for p in rng.integers(lo, hi, nb):
                dense[int(p)] = dense.get(int(p), 0) + int(rng.integers(1, 3))
            for c0 in centres:
                c = c0 + (shift_rev if strand else 0)
                for o in np.rint(rng.normal(0, sd, int(rng.integers(20, 150)))).astype(int):
                    p = c + int(o)
                    if lo <= p <= hi:
                        dense[p] = dense.get(p, 0) + 1
            if dense:
                d[name] = sorted(dense.items())
    return fwd, rev


def make_inputs(tmp_path, seed, contigs, nsamples, **kw):
    rng = np.random.default_rng(seed)
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    files = []
    for i in range(nsamples):
        fwd, rev = gen_sample(rng, contigs, **kw)
        p = tmp_path / f"s{i}.wig"
        write_wig(p, f"s{i}", fwd, rev)
        files.append(str(p))
    return str(ct), files


def run(cmd, cwd):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise AssertionError(f"{cmd[0]} failed ({r.returncode}):\n{r.stderr[-2000:]}")
    return r


def compare_tool(orc_bin, tmp_path, tool, args, outname="out.txt"):
    ref = tmp_path / ("ref_" + outname)
    got = tmp_path / ("got_" + outname)
    run([orc_bin, tool] + args + ["-o", str(ref)], tmp_path)
    run([os.path.join(BIN, tool)] + args + ["-o", str(got)], tmp_path)
    a, b = ref.read_bytes(), got.read_bytes()
    assert a == b, f"{tool} output differs\n--- oracle\n{a[:3000].decode()}\n--- bin\n{b[:3000].decode()}"
    return a.decode()


HG_LIKE = [("chrA", 60_000), ("chrB", 45_000), ("chrC", 30_000)]

REGION_CASES = [
    ("directional_basic", HG_LIKE, 1, ["-f"], {}),
    ("directional_k5_r10", HG_LIKE, 1, ["-f", "-k", "5", "-r", "10", "-t", "3"], {}),
    ("one_contig_interleave_q4", [("chrX", 80_000)], 1, ["-f"], {}),
    ("controls_prop_coeffs", HG_LIKE, 3, ["-f", "-e", "3", "-z", "p"], {}),
    ("explicit_coeffs_q6", HG_LIKE, 3, ["-e", "2", "-z", "0.7,1.3"], {}),
    ("bandwidth_20", HG_LIKE, 2, ["-f", "-b", "20"], {}),
    ("bandwidth_100", HG_LIKE, 1, ["-f", "-b", "100", "-k", "0"], {}),
    ("nondir_corr", HG_LIKE, 1, ["-D", "-y", "-f", "-s", "60"], {"shift_rev": 120}),
    ("nondir_two_samples", HG_LIKE, 2, ["-D", "-y", "-u", "0.5"], {"shift_rev": 100}),
    ("mappable_override", HG_LIKE, 1, ["-f", "-m", "3095693983"], {}),
    # outside the parallel scan: exact replay of every unit (K0)
    ("replay_threshold_zero_q11", HG_LIKE, 1, ["-f", "-r", "0"], {}),
    ("replay_negative_threshold", HG_LIKE, 2, ["-r", "-2", "-k", "0"], {}),
    ("replay_bandwidth_200", HG_LIKE, 1, ["-f", "-b", "200"], {}),
    ("replay_bandwidth_600_nondir", HG_LIKE, 1, ["-D", "-y", "-f", "-b", "600", "-u", "-1", "-r", "4",
                                                         "-k", "0"],
     {"shift_rev": 100}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", REGION_CASES, ids=lambda c: c[0])
def test_regions_cli_matches_oracle(orc_bin, gpu_lib, tmp_path, case):
    name, contigs, ns, args, kw = case
    ct, files = make_inputs(tmp_path, zlib.crc32(name.encode()) % 10_000, contigs, ns, **kw)
    out = compare_tool(orc_bin, tmp_path, "regions", ["-q", "-c", ct] + args + files)
    assert out.count("\n") > 10


PROFILE_CASES = [
    ("directional", HG_LIKE, 1, ["-f"], {}),
    ("directional_named_db", HG_LIKE, 2, ["-f", "-n", "trk", "-a", "hg19", "-b", "20"], {}),
    ("one_contig_interleave", [("chrX", 80_000)], 1, ["-f", "-b", "100"], {}),
    ("nondir", HG_LIKE, 2, ["-D", "-y"], {"shift_rev": 100}),
]


def test_oracle_profile_writer_matches_kde(orc_bin, oracle, tmp_path):
    """the oracle's -w writer (FormatOutStream::write(PosScore), format.cpp:
    1091-1132) emits exactly the nonzero KDE scores of each strand buffer,
    as %g, reverse negated, one track per strand, one variableStep per contig"""
    contigs = [("chrA", 30_000), ("chrB", 20_000)]
    rng = np.random.default_rng(5)
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    fwd, rev = gen_sample(rng, contigs)
    write_wig(tmp_path / "s0.wig", "s0", fwd, rev)
    run([orc_bin, "regions", "-q", "-f", "-c", str(ct), "-n", "trk", "-a", "hg19", "-w", "p.wig",
         "-o", "r.txt", "s0.wig"], tmp_path)
    lines = (tmp_path / "p.wig").read_text().split("\n")
    tracks = [l for l in lines if l.startswith("track")]
    assert tracks == [
        'track name="trk +" description="trk" priority=2 visibility=full type=wiggle_0 '
        'alwaysZero=on color=0,0,255 db=hg19',
        'track name="trk -" description=" " priority=2 visibility=full type=wiggle_0 '
        'alwaysZero=on color=255,0,0 altColor=255,0,0 db=hg19']
    bg = float(next(l for l in lines if l.startswith("# background=")).split("=")[1])
    got, key = {}, None
    strand = -1
    for l in lines:
        if l.startswith("track"):
            strand += 1
        elif l.startswith("variableStep"):
            key = (strand, l.split("chrom=")[1])
            assert key not in got
            got[key] = []
        elif l and not l.startswith("#"):
            got[key].append(l)
    for st, d in enumerate((fwd, rev)):
        for name, L in contigs:
            pos = np.array([p for p, _ in d[name]], np.uint32)
            cnt = np.array([[c] for _, c in d[name]], np.uint32)
            f = (oracle.profile(50, bg, L, pos, cnt) if st == 0 else
                 oracle.profile(50, bg, L, pos, None, cnt, buffer_forward=False))
            nz = np.flatnonzero(f)
            want = ["%d %s%s" % (i + 1, "-" if st else "", "%g" % f[i]) for i in nz]
            assert got[(st, name)] == want


@pytest.mark.gpu
@pytest.mark.parametrize("case", PROFILE_CASES, ids=lambda c: c[0])
def test_regions_cli_profile_matches_oracle(orc_bin, gpu_lib, tmp_path, case):
    """-w: the density profile, written in the order the reference retires
    positions (both buffers interleaved), byte-identical to the oracle's"""
    name, contigs, ns, args, kw = case
    ct, files = make_inputs(tmp_path, zlib.crc32(name.encode()) % 10_000 + 7, contigs, ns, **kw)
    common = ["-q", "-c", ct] + args
    # same file name in two directories: the default track name is its prefix
    (tmp_path / "ref").mkdir()
    (tmp_path / "got").mkdir()
    run([orc_bin, "regions"] + common + ["-w", "ref/p.wig", "-o", "ref/r.txt"] + files, tmp_path)
    run([os.path.join(BIN, "regions")] + common + ["-w", "got/p.wig", "-o", "got/r.txt"] + files,
        tmp_path)
    assert (tmp_path / "ref/r.txt").read_bytes() == (tmp_path / "got/r.txt").read_bytes()
    a, b = (tmp_path / "ref/p.wig").read_bytes(), (tmp_path / "got/p.wig").read_bytes()
    assert a.count(b"\n") > 1000
    assert a == b, "profile differs at byte %d" % next(
        (i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))


@pytest.mark.gpu
def test_regions_cli_survey_kat(orc_bin, gpu_lib, tmp_path):
    """Q7 known answer (reference run recorded in SURVEY.md) through bin/regions."""
    write_contigs(tmp_path / "ct.txt", [("chrA", 10000)])
    write_wig(tmp_path / "s1.wig", "s1", {"chrA": [(1000, 10)]}, {})
    write_wig(tmp_path / "c1.wig", "c1", {"chrA": [(1005, 7)]}, {})
    out = compare_tool(orc_bin, tmp_path, "regions",
                       ["-q", "-f", "-k", "0", "-e", "2", "-m", "1000", "-c", "ct.txt",
                        "s1.wig", "c1.wig"])
    assert out.rstrip().split("\n")[-1] == "chrA:980-1020\t1000\t-nan\t10\t0"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_strand_shift_cli_matches_oracle(orc_bin, gpu_lib, tmp_path, seed):
    contigs = [("chrA", 200_000), ("chrB", 150_000)]
    ct, files = make_inputs(tmp_path, seed, contigs, 1, shift_rev=150, n_cl=40, sd=90)
    out = compare_tool(orc_bin, tmp_path, "strand_shift",
                       ["-c", ct, "-x", "100", "-n", "10", "-u", "0", "-g", "50", "-m", "20000000"]
                       + files)
    assert "# best_shift=" in out


def test_cli_usage_errors(tmp_path):
    for tool in ("regions", "strand_shift", "tags_in_regions"):
        r = subprocess.run([os.path.join(BIN, tool)], capture_output=True, text=True)
        assert r.returncode == 1 and r.stderr.startswith("error: ")
    r = subprocess.run([os.path.join(BIN, "regions"), "--version"], capture_output=True, text=True)
    assert r.returncode == 0 and "1.0" in r.stdout


# ---- quirk Q1: tags within the first bw positions of a contig ----

@pytest.mark.gpu
@pytest.mark.parametrize("case", __import__("tests.test_oracle_kat", fromlist=["KAT"]).KAT["cases"],
                         ids=lambda c: c["name"])
def test_regions_cli_survey_kats(orc_bin, gpu_lib, tmp_path, case):
    """Every recorded reference answer (incl. both Q1 probes) through bin/regions."""
    from tests.test_oracle_kat import run_case
    _, _, rows = run_case([os.path.join(BIN, "regions")], case, tmp_path)
    got = [[r[0], int(r[1]), [int(x) for x in r[3:]]] for r in rows]
    assert got == case["expect"]


def gen_head_sample(rng, contigs, bw, tiny=()):
    """Clusters plus tags inside the first bw positions of most contigs;
    contigs named in `tiny` get tags only at positions <= bw (their buffer
    state leaks into the next contig pass)."""
    fwd, rev = gen_sample(rng, [c for c in contigs if c[1] >= 2000], lo=bw + 1, n_cl=3, sd=40)
    for d in (fwd, rev):
        for name, L in contigs:
            dense = dict(d.get(name, [])) if name not in tiny else {}
            if name in tiny or rng.random() < 0.8:
                for p in rng.integers(1, bw + 1, int(rng.integers(1, 12))):
                    dense[int(p)] = dense.get(int(p), 0) + int(rng.integers(1, 9))
            if dense:
                d[name] = sorted(dense.items())
    return fwd, rev


Q1_CASES = [
    ("dir_bw50", 50, 1, ["-f", "-k", "0"], ()),
    ("dir_bw50_leak", 50, 1, ["-f", "-k", "0"], ("c1", "c3")),
    ("dir_bw20_controls", 20, 2, ["-f", "-e", "2"], ("c2",)),
    ("dir_bw100_coeffs", 100, 3, ["-e", "3", "-z", "0.5,2", "-k", "0"], ("c1",)),
    ("nondir_bw50_corr", 50, 1, ["-D", "-y", "-f", "-k", "0"], ("c2",)),
    ("nondir_bw90_two", 90, 2, ["-D", "-f", "-k", "0"], ("c1", "c2")),
    # outside the parallel scan: the whole-buffer replay carries the leaks too
    ("replay_dir_bw200_leak", 200, 1, ["-f", "-k", "0"], ("c1",)),
    ("replay_dir_r0_leak", 50, 1, ["-f", "-k", "0", "-r", "0"], ("c3",)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", Q1_CASES, ids=lambda c: c[0])
@pytest.mark.parametrize("thr_m", ["3000", "100000"])
def test_regions_cli_q1_head_hits(orc_bin, gpu_lib, tmp_path, case, thr_m):
    name, bw, ns, args, tiny = case
    rng = np.random.default_rng(zlib.crc32((name + thr_m).encode()))
    contigs = [("c0", 9000), ("c1", 4000), ("c2", 400), ("c3", 7000), ("c4", 5000)]
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    files = []
    for i in range(ns):
        fwd, rev = gen_head_sample(rng, contigs, bw, tiny)
        p = tmp_path / f"s{i}.wig"
        write_wig(p, f"s{i}", fwd, rev)
        files.append(str(p))
    out = compare_tool(orc_bin, tmp_path, "regions",
                       ["-q", "-c", str(ct), "-b", str(bw), "-m", thr_m] + args + files)
    assert out.count("\n") > 3


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["q1_heads_bw50", "replay_bw150", "replay_r0_small"])
def test_strand_shift_cli_replayed_regions(orc_bin, gpu_lib, tmp_path, case):
    """strand_shift over regions that come from the exact replay (Q1 head
    hits, bw > 127, -r <= 0): strandCorr(shift) runs on the scores the state
    machine stored, byte-identical reports"""
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    contigs = [("c0", 60_000), ("c1", 40_000), ("c2", 30_000)]
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    bw = 150 if case == "replay_bw150" else 50
    fwd, rev = gen_sample(rng, contigs, lo=bw + 1, n_cl=12, shift_rev=40, sd=80)
    if case == "q1_heads_bw50":  # heavy stacks inside the first bw positions of every contig
        for d in (fwd, rev):
            for name, _ in contigs:
                dense = dict(d.get(name, []))
                for p in rng.integers(1, bw + 1, 8):
                    dense[int(p)] = dense.get(int(p), 0) + int(rng.integers(20, 60))
                d[name] = sorted(dense.items())
    write_wig(tmp_path / "s0.wig", "s0", fwd, rev)
    args = ["-c", str(ct), "-x", "20", "-n", "2", "-u", "-1", "-g", "30", "-m", "3000000", "-b", str(bw)]
    if case == "replay_r0_small":
        args += ["-r", "0"]
    out = compare_tool(orc_bin, tmp_path, "strand_shift", args + ["s0.wig"])
    assert "# best_shift=" in out


PROFILE_REPLAY_CASES = [
    # (name, bw, samples, args, tiny contigs)  -- units produced by the exact replay
    ("q1_heads_bw50", 50, 1, ["-f", "-k", "0"], ()),
    ("q1_leak_chain", 50, 1, ["-f", "-k", "0"], ("c1", "c3")),
    ("q1_nondir", 50, 1, ["-D", "-y", "-k", "0"], ("c2",)),
    ("whole_replay_r0", 50, 1, ["-f", "-r", "0", "-k", "0"], ()),
    ("whole_replay_bw300", 300, 2, ["-f", "-k", "0"], ("c1",)),
    ("parallel_bw200_heads", 200, 1, ["-f", "-k", "0"], ()),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", PROFILE_REPLAY_CASES, ids=lambda c: c[0])
def test_regions_cli_profile_replayed_units(orc_bin, gpu_lib, tmp_path, case):
    """-w where units come from the exact replay (quirk Q1 head hits and
    their leak chains, -r <= 0, bw > 255): the profile is written from the
    replayed state machine's own retirements (misc/peakcall.cpp:80-83), in
    the reference's order, byte-identical"""
    name, bw, ns, args, tiny = case
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    contigs = [("c0", 9000), ("c1", 4000), ("c2", 400), ("c3", 7000), ("c4", 5000)]
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    files = []
    for i in range(ns):
        fwd, rev = gen_head_sample(rng, contigs, bw, tiny)
        p = tmp_path / f"s{i}.wig"
        write_wig(p, f"s{i}", fwd, rev)
        files.append(str(p))
    common = ["-q", "-c", str(ct), "-b", str(bw), "-m", "3000"] + args
    (tmp_path / "ref").mkdir()
    (tmp_path / "got").mkdir()
    run([orc_bin, "regions"] + common + ["-w", "ref/p.wig", "-o", "ref/r.txt"] + files, tmp_path)
    run([os.path.join(BIN, "regions")] + common + ["-w", "got/p.wig", "-o", "got/r.txt"] + files, tmp_path)
    assert (tmp_path / "ref/r.txt").read_bytes() == (tmp_path / "got/r.txt").read_bytes()
    a, b = (tmp_path / "ref/p.wig").read_bytes(), (tmp_path / "got/p.wig").read_bytes()
    assert a.count(b"\n") > 100
    assert a == b, "profile differs at byte %d" % next(
        (i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
