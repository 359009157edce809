"""bin/convert_align (src/convert_align.cpp) against the
Python restatement oracle/convert_align.py: byte-identical wiggle output and
the same exit status, on generated BED, SAM, BAM (BGZF), Eland multi, Corona
and wiggle inputs -- directional and nondirectional (-D) output, shifts
(-s), read lengths (-l), the posterior filter (-p), mismatch tolerances
(-i), contigs outside the table, out-of-bounds tags, several files through
one parser, and the input errors the reference reports."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

from oracle.convert_align import convert_align as oracle_convert
from tests.wig import write_contigs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "convert_align")
TABLE = [("chrA", 30_000), ("chrB", 20_000), ("chrC", 5_000)]


def run_bin(tmp_path, files, out="out.wig", extra=()):
    r = subprocess.run([BIN, "-q", "-c", "ct.txt", "-o", out] + list(extra) + files, cwd=tmp_path,
                       capture_output=True, text=True)
    data = (tmp_path / out).read_bytes() if (tmp_path / out).exists() else None
    return r.returncode, data, r.stderr


def opts(extra):
    kw = {}
    it = iter(extra)
    for a in it:
        if a == "-D":
            kw["directional"] = False
        elif a == "-s":
            kw["offset"] = int(next(it))
        elif a == "-l":
            kw["use_len"] = int(next(it))
        elif a == "-p":
            kw["prob"] = float(next(it))
        elif a == "-i":
            kw["tol"] = int(next(it))
        elif a == "-a":
            kw["assembly"] = next(it)
        elif a == "-n":
            kw["name"] = next(it)
    return kw


def compare(tmp_path, files, extra=(), out="out.wig"):
    write_contigs(tmp_path / "ct.txt", TABLE)
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        rc, data, err = oracle_convert(TABLE, files, out, **opts(extra))
    finally:
        os.chdir(cwd)
    brc, bdata, berr = run_bin(tmp_path, files, out, extra)
    assert brc == rc, (rc, brc, err[-500:], berr[-500:])
    if rc == 0:
        assert bdata == data, f"output differs\n--- oracle\n{data[:2000]}\n--- bin\n{bdata[:2000]}"
    else:
        assert berr.strip().split("\n")[-1] == err.strip().split("\n")[-1], (err, berr)
    return data


# ---- input generators ----

def rand_aligns(rng, n, names=("chrA", "chrB", "chrC", "chrX"), maxpos=31_000):
    out = []
    for _ in range(n):
        c = names[int(rng.integers(0, len(names)))]
        out.append((c, int(rng.integers(0, maxpos)), bool(rng.random() < 0.5), int(rng.integers(20, 40))))
    return out


def write_bed(path, aligns):
    with open(path, "w") as f:
        f.write('track name="bedtrack" description="x"\n')
        for c, p, fwd, L in aligns:
            f.write(f"{c}\t{p}\t{p + L}\tread\t0\t{'+' if fwd else '-'}\n")


def sam_lines(rng, aligns):
    lines = ["@HD\tVN:1.0\tSO:unsorted", "@SQ\tSN:chrA\tLN:30000"]
    for k, (c, p, fwd, L) in enumerate(aligns):
        flag = 0 if fwd else 16
        r = rng.random()
        if r < 0.05:
            flag |= 0x100
        elif r < 0.08:
            flag |= 0x4
        elif r < 0.1:
            flag |= 0x200
        mapq = int(rng.integers(0, 60))
        tags = []
        if rng.random() < 0.7:
            tags.append(f"NM:i:{int(rng.integers(0, 4))}")
        if rng.random() < 0.3:
            tags.append("XA:Z:foo")
        seq = "".join(rng.choice(list("ACGT"), L))
        lines.append("\t".join([f"r{k}", str(flag), c, str(p), str(mapq), f"{L}M", "*", "0", "0", seq,
                                "I" * L] + tags))
    return lines


def bgzf(data):
    out = bytearray()
    for i in range(0, max(len(data), 1), 60_000):
        chunk = data[i:i + 60_000]
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = co.compress(chunk) + co.flush()
        bsize = len(comp) + 25
        out += bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", bsize)
        out += comp + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    co = zlib.compressobj(6, zlib.DEFLATED, -15)  # the BGZF end-of-file block
    comp = co.compress(b"") + co.flush()
    out += bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0]) + struct.pack("<H", len(comp) + 25)
    out += comp + struct.pack("<II", 0, 0)
    return bytes(out)


def write_bam(path, rng, aligns, refs=("chrA", "chrB", "chrC", "chrZ")):
    text = b"@HD\tVN:1.0\n"
    d = bytearray(b"BAM\1" + struct.pack("<I", len(text)) + text + struct.pack("<I", len(refs)))
    for r in refs:
        nm = r.encode() + b"\0"
        d += struct.pack("<I", len(nm)) + nm + struct.pack("<I", 100_000)
    for k, (c, p, fwd, L) in enumerate(aligns):
        rid = refs.index(c) if c in refs else -1
        flag = (0 if fwd else 16)
        r = rng.random()
        if r < 0.05:
            flag |= 0x100
        elif r < 0.08:
            flag |= 0x4
        name = f"q{k}".encode() + b"\0"
        cigar = struct.pack("<I", (L << 4) | 0)
        seq = bytes((L + 1) // 2)
        qual = bytes([30] * L)
        tags = b""
        t = rng.random()
        if t < 0.4:
            tags += b"NMC" + bytes([int(rng.integers(0, 4))])
        elif t < 0.6:
            tags += b"XZZhello\0" + b"NMi" + struct.pack("<i", int(rng.integers(0, 4)))
        elif t < 0.7:
            tags += b"NMs" + struct.pack("<h", int(rng.integers(0, 4)))
        mapq = int(rng.integers(0, 60))
        core = struct.pack("<iiIIiiii", rid, p, (mapq << 8) | len(name), (flag << 16) | 1, L, -1, -1, 0)
        rec = core + name + cigar + seq + qual + tags
        d += struct.pack("<I", len(rec)) + rec
    open(path, "wb").write(bgzf(bytes(d)))


def write_wig_in(path, rng, directional=True):
    with open(path, "w") as f:
        f.write("# tags=0\n")
        strands = ("+", "-") if directional else (None,)
        for st in strands:
            nm = f"w {st}" if st else "w"
            f.write(f'track name="{nm}" description="d" type=wiggle_0\n')
            for c in ("chrB", "chrQ", "chrA"):
                f.write(f"variableStep chrom={c}\n")
                for p in sorted(set(int(x) for x in rng.integers(1, 21_000, 300))):
                    k = int(rng.integers(1, 9))
                    f.write(f"{p} {'-' if st == '-' else ''}{k}\n")


def eland_lines(rng, n, L=25):
    out = []
    for k in range(n):
        seq = "".join(rng.choice(list("ACGTN" if rng.random() < 0.1 else "ACGT"), L))
        kind = rng.random()
        if kind < 0.1:
            out.append(f">r{k}\t{seq}\tNM\t-")
            continue
        c0, c1, c2 = (int(rng.integers(0, 2)), int(rng.integers(0, 3)), int(rng.integers(0, 5)))
        hits = []
        nh = max(1, c0 + c1 + c2)
        for h in range(min(nh, 3)):
            contig = ["chrA.fa", "chrB.fa", "x/chrC.fa", "chrQ.fa"][int(rng.integers(0, 4))]
            pos = int(rng.integers(1, 28_000))
            d = "F" if rng.random() < 0.5 else "R"
            mm = ["", "0", "1", "2", "12A", "5C3G"][int(rng.integers(0, 6))] or str(int(rng.integers(0, 3)))
            hits.append((f"{contig}:" if h == 0 or rng.random() < 0.5 else "") + f"{pos}{d}{mm}")
        out.append(f">r{k}\t{seq}\t{c0}:{c1}:{c2}\t{','.join(hits)}")
    return out


def corona_lines(rng, n, L=25):
    out = ["# corona"]
    for k in range(n):
        hits = []
        for _ in range(int(rng.integers(0, 4))):
            c = ["chrA", "chrB", "chrC", "chrQ"][int(rng.integers(0, 4))]
            p = int(rng.integers(0, 28_000))
            hits.append(f"{c}.{'-' if rng.random() < 0.5 else ''}{p}.{int(rng.integers(0, 3))}")
        out.append(f">{k}_{k + 1}_{k + 2}_F3" + ("," + ",".join(hits) if hits else ""))
        out.append("T" + "".join(rng.choice(list("0123"), L)))
    return out


# ---- tests ----

@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["-D"], ["-s", "30"], ["-s", "-25", "-D"], ["-l", "30"],
                                   ["-p", "0", "-a", "hg19", "-n", "myname"]])
def test_convert_bed_sam(gpu_lib, tmp_path, extra):
    rng = np.random.default_rng(1)
    write_bed(tmp_path / "a.bed", rand_aligns(rng, 3000))
    (tmp_path / "b.sam").write_text("\n".join(sam_lines(rng, rand_aligns(rng, 3000))) + "\n")
    compare(tmp_path, ["a.bed", "b.sam"], extra)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["-D"], ["-i", "3", "-p", "0"], ["-p", "0.5", "-s", "10"]])
def test_convert_bam(gpu_lib, tmp_path, extra):
    rng = np.random.default_rng(2)
    write_bam(tmp_path / "a.bam", rng, rand_aligns(rng, 5000, names=("chrA", "chrB", "chrC", "chrZ")))
    compare(tmp_path, ["a.bam"], extra)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["-D"], ["-p", "0"], ["-l", "20"], ["-i", "0"]])
def test_convert_eland_corona(gpu_lib, tmp_path, extra):
    rng = np.random.default_rng(3)
    (tmp_path / "a.txt").write_text("\n".join(eland_lines(rng, 2000)) + "\n")
    (tmp_path / "b.csfasta").write_text("\n".join(corona_lines(rng, 2000)) + "\n")
    compare(tmp_path, ["a.txt", "b.csfasta"], extra)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["-D"], ["-l", "10", "-s", "5"]])
def test_convert_wiggle_inputs(gpu_lib, tmp_path, extra):
    rng = np.random.default_rng(4)
    write_wig_in(tmp_path / "d.wig", rng, True)
    write_wig_in(tmp_path / "n.wig", rng, False)
    compare(tmp_path, ["d.wig", "n.wig"], extra)


@pytest.mark.gpu
def test_convert_errors(gpu_lib, tmp_path):
    rng = np.random.default_rng(5)
    (tmp_path / "bad.sam").write_text("\n".join(sam_lines(rng, rand_aligns(rng, 50)) + ["r\tx\tchrA"]) + "\n")
    compare(tmp_path, ["bad.sam"])
    (tmp_path / "none.bed").write_text("chrQ\t10\t40\tr\t0\t+\n")
    compare(tmp_path, ["none.bed"])  # nothing to do
    (tmp_path / "what.txt").write_text("hello world\n")
    compare(tmp_path, ["what.txt"])  # unknown format
    # two Eland files with different read lengths: the read length carries over
    (tmp_path / "e1.txt").write_text(">a\tACGTACGTAC\t1:0:0\tchrA.fa:100F0\n")
    (tmp_path / "e2.txt").write_text(">b\tACGTACGTACGT\t1:0:0\tchrA.fa:200F0\n")
    compare(tmp_path, ["e1.txt", "e2.txt"], ["-p", "0"])


@pytest.mark.gpu
def test_convert_large_count_map(gpu_lib, tmp_path):
    """many alignments at few positions (per-position sums), both strands,
    every contig edge (positions 1 and the contig length)"""
    rng = np.random.default_rng(6)
    al = []
    for c, L in TABLE:
        for p in (0, L - 30, 7, 7, 7):
            for fwd in (True, False):
                al.append((c, p, fwd, 30))
    al += rand_aligns(rng, 20_000, names=("chrA",), maxpos=200)
    write_bed(tmp_path / "x.bed", al)
    compare(tmp_path, ["x.bed"])
    compare(tmp_path, ["x.bed"], ["-D"], out="nd.wig")


def test_oracle_convert_known_answer(tmp_path):
    """the restatement on a hand-checked case: BED is 0-based half-open; the
    reverse tag sits at its 5' end (the BED end); -D merges strands"""
    (tmp_path / "k.bed").write_text("chrA\t99\t125\tr\t0\t+\nchrA\t99\t125\tr\t0\t+\n"
                                    "chrA\t200\t226\tr\t0\t-\nchrB\t0\t26\tr\t0\t+\n")
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        rc, out, _ = oracle_convert(TABLE, ["k.bed"], "k.wig", prob=0)
        rc2, out2, _ = oracle_convert(TABLE, ["k.bed"], "k.wig", directional=False, prob=0)
    finally:
        os.chdir(cwd)
    assert rc == 0 and rc2 == 0
    assert out.decode().split("\n")[2:] == [
        'track name="k +" description="k" priority=3 visibility=full type=wiggle_0 alwaysZero=on color=0,0,255',
        "variableStep chrom=chrA", "100 2", "variableStep chrom=chrB", "1 1",
        'track name="k -" description=" " priority=3 visibility=full type=wiggle_0 alwaysZero=on '
        'color=255,0,0 altColor=255,0,0',
        "variableStep chrom=chrA", "226 -1", ""]
    assert out2.decode().split("\n")[3:] == ["variableStep chrom=chrA", "100 2", "226 1",
                                             "variableStep chrom=chrB", "1 1", ""]


def test_convert_align_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    write_contigs(tmp_path / "ct.txt", TABLE)
    (tmp_path / "k.bed").write_text("chrA\t99\t125\tr\t0\t+\n")
    r = subprocess.run([BIN, "-q", "-c", "ct.txt", "-o", "o.wig", "k.bed"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_count_map_device_order(gpu_lib):
    """up_cm_* through the C-ABI against dictionaries: per-position sums with
    uint32 wrap, both iterators' orders, contig edges, an invalid add"""
    rng = np.random.default_rng(7)
    lens = [1, 70_000, 8_191, 8_193, 100]
    n = 200_000
    c = rng.integers(0, len(lens), n).astype(np.uint32)
    p = np.array([int(rng.integers(1, lens[k] + 1)) for k in c], np.uint32)
    f = (rng.random(n) < 0.5).astype(np.uint8)
    k = rng.integers(1, 5, n).astype(np.uint32)
    k[:3] = 0xFFFFFFFF
    with gpu_lib.CountMap(lens) as cm:
        cm.add(c, p, f, k)
        cm.add(c[:1000], p[:1000], f[:1000])  # count NULL: 1 each
        with pytest.raises(gpu_lib.UpError):
            cm.add([1], [lens[1] + 1], [1])
        d_dir = cm.collect(False)
        d_nd = cm.collect(True)
    want = {}
    for i in range(n):
        key = (int(f[i] == 0), int(c[i]), int(p[i]))
        want[key] = (want.get(key, 0) + int(k[i])) & 0xFFFFFFFF
    for i in range(1000):
        key = (int(f[i] == 0), int(c[i]), int(p[i]))
        want[key] = (want.get(key, 0) + 1) & 0xFFFFFFFF
    exp = sorted((s, cc, pp, v) for (s, cc, pp), v in want.items() if v)
    got = [(int(1 - ff), int(cc), int(pp), int(v)) for cc, pp, v, ff in zip(*d_dir)]
    assert got == exp
    nd = {}
    for (s, cc, pp), v in want.items():
        nd[(cc, pp)] = (nd.get((cc, pp), 0) + v) & 0xFFFFFFFF
    exp_nd = sorted((cc, pp, v) for (cc, pp), v in nd.items() if v)
    assert [(int(cc), int(pp), int(v)) for cc, pp, v, _ in zip(*d_nd)] == exp_nd
    assert d_nd[3].all()
