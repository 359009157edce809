"""gzip / bzip2 stream filters at the boundary (misc/filterstream.cpp:30-50,
86-104: a file name ending in ".gz" is read and written through gzip filters,
".bz2" through bzip2 ones).  The canonical pipeline always gzips its wiggle
files (generate_script.pl:7, 255-276): convert_align -o x.wig.gz, then
strand_shift and regions -D -s on the .wig.gz files.  libbz2's headers are
absent here, so ".bz2" is refused with an "error:" line and exit 1 on both
ends (never read or written as plain bytes).

CPU part: the oracle CLI's filters.  GPU part: the same pipeline through
bin/ against the oracle, byte-identical after decompression."""
import gzip
import os
import subprocess

import numpy as np
import pytest

from tests.test_cli import gen_sample, run
from tests.wig import write_contigs, write_wig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")
CONTIGS = [("chrA", 60_000), ("chrB", 45_000), ("chrC", 30_000)]


def _inputs(tmp_path, seed=3, n=2, shift_rev=0):
    rng = np.random.default_rng(seed)
    write_contigs(tmp_path / "ct.txt", CONTIGS)
    plain = []
    for i in range(n):
        fwd, rev = gen_sample(rng, CONTIGS, shift_rev=shift_rev)
        p = tmp_path / f"s{i}.wig"
        write_wig(p, f"s{i}", fwd, rev)
        with open(p, "rb") as f, gzip.open(str(p) + ".gz", "wb") as g:  # Python's gzip module
            g.write(f.read())
        plain.append(p.name)
    return plain


def _table_body(path):
    data = gzip.open(path).read() if str(path).endswith(".gz") else open(path, "rb").read()
    # "# align_file=<name>" carries the input's file name; everything else must agree
    return b"\n".join(l for l in data.split(b"\n") if not l.startswith(b"# align_file="))


def test_oracle_reads_and_writes_gz(orc_bin, tmp_path):
    plain = _inputs(tmp_path)
    gz = [p + ".gz" for p in plain]
    run([orc_bin, "regions", "-q", "-f", "-c", "ct.txt", "-o", "a.txt"] + plain, tmp_path)
    run([orc_bin, "regions", "-q", "-f", "-c", "ct.txt", "-o", "b.txt.gz"] + gz, tmp_path)
    b = (tmp_path / "b.txt.gz").read_bytes()
    assert b[:2] == b"\x1f\x8b"  # a gzip stream, not plain text under a .gz name
    assert _table_body(tmp_path / "a.txt") == _table_body(tmp_path / "b.txt.gz")
    assert b"# align_file=s0.wig.gz" in gzip.decompress(b)
    rows = [l for l in _table_body(tmp_path / "a.txt").split(b"\n") if l.startswith(b"chr")]
    assert len(rows) > 10


@pytest.mark.parametrize("where", ["input", "output"])
def test_oracle_refuses_bz2(orc_bin, tmp_path, where):
    plain = _inputs(tmp_path, n=1)
    if where == "input":
        (tmp_path / "s0.wig.bz2").write_bytes((tmp_path / plain[0]).read_bytes())
        args, out = ["s0.wig.bz2"], "o.txt"
    else:
        args, out = plain, "o.txt.bz2"
    r = subprocess.run([orc_bin, "regions", "-q", "-c", "ct.txt", "-o", out] + args, cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 1 and "error:" in r.stderr and "bz2" in r.stderr
    assert not (tmp_path / "o.txt.bz2").exists()


def test_oracle_refuses_plain_bytes_named_gz(orc_bin, tmp_path):
    """boost's gzip_decompressor throws on a missing gzip header; zlib's
    transparent mode would read the file as plain text -- refused instead"""
    plain = _inputs(tmp_path, n=1)
    (tmp_path / "s0.wig.gz").write_bytes((tmp_path / plain[0]).read_bytes())
    r = subprocess.run([orc_bin, "regions", "-q", "-c", "ct.txt", "-o", "o.txt", "s0.wig.gz"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 1 and "not in gzip format" in r.stderr, r.stderr[-300:]


# ---- bin/ (GPU) --------------------------------------------------------------

def _same(orc_bin, tmp_path, tool, args, out):
    run([orc_bin, tool] + args + ["-o", "ref_" + out], tmp_path)
    run([os.path.join(BIN, tool)] + args + ["-o", "got_" + out], tmp_path)
    a, b = (tmp_path / ("ref_" + out)).read_bytes(), (tmp_path / ("got_" + out)).read_bytes()
    if out.endswith(".gz"):
        assert a[:2] == b[:2] == b"\x1f\x8b"
        a, b = gzip.decompress(a), gzip.decompress(b)
    assert a == b, f"{tool}: outputs differ"
    return a.decode()


@pytest.mark.gpu
def test_pipeline_on_gzipped_wiggles(orc_bin, gpu_lib, tmp_path):
    """generate_script.pl's shell script on .wig.gz files: strand_shift
    then regions -D -s <best> (+ -w profile.wig.gz) and tags_in_regions, bin/
    against the oracle, every output gzipped and identical after
    decompression; and bin/ on .wig.gz equals bin/ on the plain files"""
    plain = _inputs(tmp_path, n=2, shift_rev=150)
    gz = [p + ".gz" for p in plain]
    rep = _same(orc_bin, tmp_path, "strand_shift", ["-x", "100", "-c", "ct.txt", gz[0]], "shift.txt.gz")
    best = [l for l in rep.splitlines() if l.startswith("# best_shift=")][0].split("=")[1]
    args = ["-D", "-y", "-u", "-1", "-r", "5", "-s", best, "-c", "ct.txt"]
    _same(orc_bin, tmp_path, "regions", args + ["-w", "prof.wig.gz"] + gz, "regions.txt.gz")
    table = _same(orc_bin, tmp_path, "regions", args + gz, "r2.txt.gz")
    assert sum(1 for l in table.splitlines() if l.startswith("chr")) > 10
    run([os.path.join(BIN, "regions")] + args + ["-o", "plain.txt"] + plain, tmp_path)
    assert _table_body(tmp_path / "plain.txt") == _table_body(tmp_path / "got_r2.txt.gz")
    _same(orc_bin, tmp_path, "tags_in_regions", ["-D", "-c", "ct.txt", "-f", "got_r2.txt.gz"] + gz,
          "tir.txt.gz")


@pytest.mark.gpu
def test_profile_output_gzipped(orc_bin, gpu_lib, tmp_path):
    """-w x.wig.gz: the density profile through the gzip filter"""
    plain = _inputs(tmp_path, n=1)
    for tool, who in ((orc_bin, "ref"), (os.path.join(BIN, "regions"), "got")):
        (tmp_path / who).mkdir()  # same file names: the profile's track name is its file name's prefix
        cmd = [tool] + (["regions"] if tool == orc_bin else [])
        run(cmd + ["-f", "-c", "../ct.txt", "-w", "p.wig.gz", "-o", "t.txt", "../" + plain[0]],
            tmp_path / who)
    a, b = ((tmp_path / w / "p.wig.gz").read_bytes() for w in ("ref", "got"))
    assert b[:2] == b"\x1f\x8b"
    assert gzip.decompress(a) == gzip.decompress(b) and len(gzip.decompress(b)) > 1000


@pytest.mark.gpu
def test_convert_align_writes_gzip(gpu_lib, tmp_path):
    """convert_align -o x.wig.gz (the pipeline's first step): a gzip stream
    whose content is the plain -o output; regions reads it back"""
    rng = np.random.default_rng(5)
    write_contigs(tmp_path / "ct.txt", CONTIGS)
    with open(tmp_path / "a.bed", "w") as f:
        for _ in range(20_000):
            c, L = CONTIGS[int(rng.integers(0, 3))]
            s = int(rng.integers(0, L - 40))
            f.write(f"{c}\t{s}\t{s + 36}\tr\t0\t{'+-'[int(rng.integers(0, 2))]}\n")
    ca = os.path.join(BIN, "convert_align")
    run([ca, "-q", "-c", "ct.txt", "-o", "x.wig", "a.bed"], tmp_path)
    run([ca, "-q", "-c", "ct.txt", "-o", "x.wig.gz", "a.bed"], tmp_path)
    z = (tmp_path / "x.wig.gz").read_bytes()
    assert z[:2] == b"\x1f\x8b" and gzip.decompress(z) == (tmp_path / "x.wig").read_bytes()
    run([os.path.join(BIN, "regions"), "-q", "-c", "ct.txt", "-r", "2", "-o", "r.txt", "x.wig.gz"],
        tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("tool", ["regions", "strand_shift", "convert_align", "tags_in_regions"])
@pytest.mark.parametrize("where", ["input", "output"])
def test_bin_refuses_bz2(gpu_lib, tmp_path, tool, where):
    plain = _inputs(tmp_path, n=1)
    (tmp_path / "s0.wig.bz2").write_bytes((tmp_path / plain[0]).read_bytes())
    orc = os.path.join(ROOT, "oracle", "_build", "orc")
    run([orc, "regions", "-q", "-c", "ct.txt", "-o", "reg.txt", plain[0]], tmp_path)
    inp = "s0.wig.bz2" if where == "input" else plain[0]
    out = "o.txt" if where == "input" else "o.txt.bz2"
    extra = {"tags_in_regions": ["-f", "reg.txt"], "strand_shift": ["-x", "20", "-u", "-1"]}.get(tool, [])
    quiet = ["-q"] if tool in ("regions", "convert_align") else []  # the CLIs that take -q
    r = subprocess.run([os.path.join(BIN, tool)] + quiet + ["-c", "ct.txt", "-o", out] + extra + [inp],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 1 and "error:" in r.stderr and "bz2" in r.stderr, r.stderr[-500:]
    assert not (tmp_path / "o.txt.bz2").exists() or (tmp_path / "o.txt.bz2").stat().st_size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("tool", ["regions", "tags_in_regions"])
def test_bin_refuses_plain_bytes_named_gz(gpu_lib, tmp_path, tool):
    plain = _inputs(tmp_path, n=1)
    (tmp_path / "s0.wig.gz").write_bytes((tmp_path / plain[0]).read_bytes())
    orc = os.path.join(ROOT, "oracle", "_build", "orc")
    run([orc, "regions", "-q", "-c", "ct.txt", "-o", "reg.txt", plain[0]], tmp_path)
    extra = {"tags_in_regions": ["-f", "reg.txt"]}.get(tool, [])
    quiet = ["-q"] if tool == "regions" else []
    r = subprocess.run([os.path.join(BIN, tool)] + quiet + ["-c", "ct.txt", "-o", "o.txt"] + extra + ["s0.wig.gz"],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 1 and "not in gzip format" in r.stderr, r.stderr[-500:]
