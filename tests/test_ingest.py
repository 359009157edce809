"""Host ingest on CPU: the lexed, multi-threaded wiggle
reader and the per-iteration parallel merge must build exactly the units,
event clocks and stream counters of the plain serial replay of the
reference's loop (src/regions.cpp:311-391) -- and fail with the same error
message where the input is bad.

bin/regions and bin/strand_shift stop before the GPU phase when
UNIPEAK_DUMP_UNITS names a file; UNIPEAK_SERIAL_INGEST=1 selects the serial
merge and UNIPEAK_NO_LEX=1 the getline reader."""
import os
import subprocess

import numpy as np
import pytest

from tests.test_cli import BIN, gen_sample
from tests.wig import write_contigs, write_wig

MODES = {
    "plain_serial": {"UNIPEAK_NO_LEX": "1", "UNIPEAK_SERIAL_INGEST": "1"},
    "lexed_serial": {"UNIPEAK_SERIAL_INGEST": "1"},
    "lexed_parallel": {"UNIPEAK_THREADS": "4"},
    "lexed_parallel_1": {"UNIPEAK_THREADS": "1"},
    "lexed_parallel_small_chunks": {"UNIPEAK_THREADS": "3", "UNIPEAK_LEX_CHUNK": "1500"},
}


def dump(tmp_path, tool, args, mode):
    out = tmp_path / f"dump_{mode}.txt"
    env = dict(os.environ, UNIPEAK_DUMP_UNITS=str(out), **MODES[mode])
    r = subprocess.run([os.path.join(BIN, tool)] + args, cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=120)
    text = out.read_text() if out.exists() else ""
    if out.exists():
        out.unlink()
    path = [l for l in text.split("\n") if l.startswith("ingest ")]
    dump.paths[mode] = path[0].split()[1] if path else None
    text = "\n".join(l for l in text.split("\n") if not l.startswith("ingest "))
    return r.returncode, r.stderr, text


dump.paths = {}


def same_everywhere(tmp_path, tool, args, parallel=True):
    """every mode gives the serial replay's result; `parallel` says whether
    the parallel merge should have handled the input (else it must defer)"""
    ref = dump(tmp_path, tool, args, "plain_serial")
    for mode in MODES:
        if mode != "plain_serial":
            got = dump(tmp_path, tool, args, mode)
            assert got == ref, f"{mode} differs from the serial replay\n{ref[1]}\n{got[1]}"
    if ref[0] == 0:
        assert dump.paths["lexed_parallel"] == ("parallel" if parallel else "serial")
    return ref


CONTIGS = [("chrA", 40_000), ("chrB", 25_000), ("chrC", 12_000)]


def inputs(tmp_path, n, seed=3, contigs=CONTIGS, **kw):
    rng = np.random.default_rng(seed)
    write_contigs(tmp_path / "ct.txt", contigs)
    files = []
    for i in range(n):
        fwd, rev = gen_sample(rng, contigs, **kw)
        write_wig(tmp_path / f"s{i}.wig", f"s{i}", fwd, rev)
        files.append(f"s{i}.wig")
    return files


@pytest.mark.parametrize("flags,n,kw", [
    (["-f"], 1, {}),
    (["-f", "-e", "3"], 3, {}),
    (["-D", "-y"], 2, {"shift_rev": 100}),
    (["-f", "-s", "40", "-l", "30"], 2, {}),
    (["-f", "-b", "20"], 1, {"lo": 5}),  # head hits (quirk Q1) reach the units
])
def test_regions_ingest_modes_agree(tmp_path, flags, n, kw):
    files = inputs(tmp_path, n, **kw)
    rc, err, text = same_everywhere(tmp_path, "regions", ["-q", "-c", "ct.txt", "-o", "o.txt"]
                                    + flags + files)
    assert rc == 0 and text.count("unit ") >= 3


def test_single_contig_interleave_q4(tmp_path):
    files = inputs(tmp_path, 2, contigs=[("chrX", 50_000)])
    rc, _, text = same_everywhere(tmp_path, "regions", ["-q", "-f", "-c", "ct.txt", "-o", "o.txt"]
                                  + files)
    assert rc == 0
    # the reverse track is consumed in the forward pass: both buffers in iteration 0
    assert "unit b1 c0 it0" in text


def test_strand_shift_ingest_modes_agree(tmp_path):
    files = inputs(tmp_path, 1, shift_rev=120)
    rc, _, _ = same_everywhere(tmp_path, "strand_shift", ["-c", "ct.txt"] + files)
    assert rc == 0


def write_raw(path, lines, trailing_newline=True):
    text = "\n".join(lines) + ("\n" if trailing_newline else "")
    path.write_bytes(text.encode())


HDR_F = ('track name="x +" description="x" priority=3 visibility=full type=wiggle_0 '
         'alwaysZero=on color=0,0,255')
HDR_R = ('track name="x -" description=" " priority=3 visibility=full type=wiggle_0 '
         'alwaysZero=on color=255,0,0 altColor=255,0,0')


def data(rng, lo, hi, n, neg=False):
    pos = np.unique(rng.integers(lo, hi, n))
    return [f"{p} {'-' if neg else ''}{int(rng.integers(1, 4))}" for p in pos]


def test_stream_out_of_table_order_and_unknown_contigs(tmp_path):
    """a wig listing chrB before chrA, plus a contig missing from the table:
    runs the merge never reaches leave the stream stuck (serial replay)"""
    rng = np.random.default_rng(8)
    write_contigs(tmp_path / "ct.txt", CONTIGS)
    lines = ["# tags=900", HDR_F, "variableStep chrom=chrB"] + data(rng, 300, 20_000, 200)
    lines += ["variableStep chrom=chrZ"] + data(rng, 300, 20_000, 50)
    lines += ["variableStep chrom=chrA"] + data(rng, 300, 30_000, 200)
    lines += [HDR_R, "variableStep chrom=chrA"] + data(rng, 300, 30_000, 200, True)
    lines += ["variableStep chrom=chrC"] + data(rng, 300, 10_000, 100, True)
    lines += ["variableStep chrom=chrB"] + data(rng, 300, 20_000, 100, True)  # never reached
    write_raw(tmp_path / "s0.wig", lines)
    rc, _, text = same_everywhere(tmp_path, "regions", ["-q", "-f", "-c", "ct.txt", "-o", "o.txt",
                                                        "s0.wig"], parallel=False)
    assert rc == 0 and "unit b0 c1 it1" in text


@pytest.mark.parametrize("case", ["bad_line", "crlf", "no_tags_header", "no_trailing_newline",
                                  "out_of_bounds", "huge_values", "comments_blank"])
def test_line_grammar_edges(tmp_path, case):
    rng = np.random.default_rng(11)
    write_contigs(tmp_path / "ct.txt", CONTIGS)
    body = [HDR_F, "variableStep chrom=chrA"] + data(rng, 300, 30_000, 300)
    body += ["variableStep chrom=chrB"] + data(rng, 300, 20_000, 200)
    body += [HDR_R, "variableStep chrom=chrA"] + data(rng, 300, 30_000, 300, True)
    head = ["# tags=1000"]
    trailing = True
    if case == "bad_line":
        body.insert(200, "1234 x5")
    elif case == "crlf":
        body = [l + "\r" if l[0].isdigit() else l for l in body]
    elif case == "no_tags_header":
        head = ["# made by hand"]
    elif case == "no_trailing_newline":
        trailing = False
    elif case == "out_of_bounds":
        body.insert(100, "0 4")
        body.insert(150, "39999 2")
        body.insert(151, "40001 2")
        body.insert(260, "99999999999 1")
    elif case == "huge_values":
        body.insert(50, "4294967295 1")
        body.insert(51, "4294967296 1")
        body.insert(120, "00000000000123 7")
        body.insert(121, "123\t\t7")
        body.insert(122, "123 -4294967295")
    elif case == "comments_blank":
        body.insert(30, "")
        body.insert(31, "# comment 5 5")
        body.insert(90, "  ")
    write_raw(tmp_path / "s0.wig", head + body, trailing)
    rc, err, _ = same_everywhere(tmp_path, "regions", ["-q", "-f", "-c", "ct.txt", "-o", "o.txt",
                                                       "s0.wig"])
    if case in ("bad_line", "crlf"):
        assert rc == 1 and "bad format" in err


def test_nondir_out_of_order_error(tmp_path):
    rng = np.random.default_rng(12)
    write_contigs(tmp_path / "ct.txt", CONTIGS)
    fwd = data(rng, 300, 30_000, 300)
    fwd[150], fwd[151] = fwd[151], fwd[150]
    write_raw(tmp_path / "s0.wig", ["# tags=700", HDR_F, "variableStep chrom=chrA"] + fwd
              + [HDR_R, "variableStep chrom=chrA"] + data(rng, 300, 30_000, 300, True))
    rc, err, _ = same_everywhere(tmp_path, "regions", ["-q", "-D", "-c", "ct.txt", "-o", "o.txt",
                                                       "s0.wig"])
    assert rc == 1 and "alignments out of order" in err
