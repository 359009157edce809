"""bin/wigs2bigwigs (the native replacement of extras/wigs2bigwigs.pl +
UCSC wigToBigWig -clip): the bigWig files are decoded with
an independent reader of the BBI layout (header, chromosome B+ tree, R-tree
index, zlib sections) and must hold exactly the intervals and float32 values
of the wiggle input (clipped at the chromosome ends), and the printed track
headers must be the script's.  Host-only: runs on CPU.

Parity note: wigToBigWig is not in this image, so the files are checked for
content, not bytes (its section sizes and zoom levels are its own)."""
import os
import re
import struct
import subprocess
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin", "wigs2bigwigs")


def read_bigwig(path):
    """{chrom: [(start, end, value)]} through the R-tree, plus the header"""
    b = open(path, "rb").read()
    magic, ver, zooms, ctree, data, index, fc, dfc, asq, tsum, ubuf, ext = struct.unpack_from(
        "<IHHQQQHHQQIQ", b, 0)
    assert magic == 0x888FFC26 and ver == 4
    assert struct.unpack_from("<I", b, len(b) - 4)[0] == 0x888FFC26
    bm, bsize, ksize, vsize, nitems, _ = struct.unpack_from("<IIIIQQ", b, ctree)
    assert bm == 0x78CA8C91 and vsize == 8
    chroms = {}

    def walk_b(off):
        leaf, _, cnt = struct.unpack_from("<BBH", b, off)
        off += 4
        for _ in range(cnt):
            key = b[off:off + ksize].rstrip(b"\0").decode()
            if leaf:
                cid, size = struct.unpack_from("<II", b, off + ksize)
                chroms[cid] = (key, size)
                off += ksize + 8
            else:
                child, = struct.unpack_from("<Q", b, off + ksize)
                walk_b(child)
                off += ksize + 8
    walk_b(ctree + 32)
    assert len(chroms) == nitems
    names = [chroms[i][0] for i in range(len(chroms))]
    assert names == sorted(names)  # ids in key order
    rm, rbs, ritems, sc, sb, ec, eb, efo, ips, _ = struct.unpack_from("<IIQIIIIQII", b, index)
    assert rm == 0x2468ACE0
    assert struct.unpack_from("<Q", b, data)[0] == ritems
    blocks = []

    def walk_r(off):
        leaf, _, cnt = struct.unpack_from("<BBH", b, off)
        off += 4
        for _ in range(cnt):
            if leaf:
                blocks.append(struct.unpack_from("<IIIIQQ", b, off))
                off += 32
            else:
                walk_r(struct.unpack_from("<IIIIQ", b, off)[4])
                off += 24
    walk_r(index + 48)
    assert len(blocks) == ritems
    out = {}
    for c0, s0, c1, s1, doff, dsize in blocks:
        raw = zlib.decompress(b[doff:doff + dsize]) if ubuf else b[doff:doff + dsize]
        assert len(raw) <= ubuf
        cid, cs, ce, step, span, typ, _, n = struct.unpack_from("<IIIIIBBH", raw, 0)
        assert (cid, cs) == (c0, s0) and c0 == c1 and ce == s1
        p = 24
        for k in range(n):
            if typ == 1:
                s, e, v = struct.unpack_from("<IIf", raw, p)
                p += 12
            elif typ == 2:
                s, v = struct.unpack_from("<If", raw, p)
                e = s + span
                p += 8
            else:
                v, = struct.unpack_from("<f", raw, p)
                s = cs + k * step
                e = s + span
                p += 4
            out.setdefault(chroms[cid][0], []).append((s, e, v))
    return out, chroms


def expected(path, sizes):
    """the wiggle's tracks as the script splits them: [(strand, {chrom: items})]"""
    tracks, chrom, span = [], None, 1
    for line in open(path):
        if line.startswith("#"):
            continue
        if line.startswith("track"):
            m = re.search(r'name=".+([+-])"', line)
            tracks.append((m.group(1) if m else "", {}))
            continue
        line = line.strip()
        if not line:
            continue
        if line.startswith("variableStep"):
            chrom = re.search(r"chrom=(\S+)", line).group(1)
            m = re.search(r"span=(\d+)", line)
            span = int(m.group(1)) if m else 1
            continue
        p, v = line.split()
        s, e = int(p) - 1, int(p) - 1 + span
        if s >= sizes[chrom]:
            continue
        e = min(e, sizes[chrom])
        tracks[-1][1].setdefault(chrom, []).append((s, e, float(np.float32(float(v)))))
    for _, d in tracks:
        for c in d:
            d[c].sort(key=lambda t: t[0])
    return tracks


def test_wigs2bigwigs_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    sizes = {"chr1": 300_000, "chr2": 120_000, "chrM": 16_571}
    (tmp_path / "s.sizes").write_text("".join(f"{c}\t{L}\n" for c, L in sizes.items()))
    with open(tmp_path / "p.wig", "w") as f:  # a -w density profile: both strands
        f.write("# original_file=x\n")
        for strand, name in (("+", "prof +"), ("-", "prof -")):
            f.write(f'track name="{name}" description="d" priority=2 visibility=full type=wiggle_0 '
                    'alwaysZero=on color=0,0,255\n')
            for c in ("chr2", "chr1", "chrM"):
                f.write(f"variableStep chrom={c}\n")
                pos = np.unique(rng.integers(1, sizes[c] + 40, 3000))  # some past the end (-clip)
                for p in pos:
                    v = float(rng.random() * 50)
                    f.write(f"{p} {'-' if strand == '-' else ''}{v:.6g}\n")
    r = subprocess.run([BIN, "--sizes", "s.sizes", "--prefix", "http://h/", "p.wig"], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    hdr = r.stdout.strip().split("\n")
    assert hdr[0].startswith('track name="prof +"') and "type=bigWig" in hdr[0]
    assert hdr[0].endswith(" bigDataUrl=http://h/p+.bw") and hdr[1].endswith(" bigDataUrl=http://h/p-.bw")
    want = expected(tmp_path / "p.wig", sizes)
    for strand, items in want:
        got, chroms = read_bigwig(tmp_path / f"p{strand}.bw")
        assert {v[0]: v[1] for v in chroms.values()} == {c: sizes[c] for c in items}
        assert set(got) == set(items)
        for c in items:
            assert got[c] == items[c], c


def test_wigs2bigwigs_errors(tmp_path):
    (tmp_path / "s.sizes").write_text("chr1\t1000\n")
    (tmp_path / "a.wig").write_text("variableStep chrom=chr1\n5 1\n")
    r = subprocess.run([BIN, "--sizes", "s.sizes", "a.wig"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode != 0 and "error: no track defined at line 1" in r.stderr
    (tmp_path / "b.wig").write_text('track name="b" type=wiggle_0\nvariableStep chrom=chrQ\n5 1\n')
    r = subprocess.run([BIN, "--sizes", "s.sizes", "b.wig"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode != 0 and "chrQ" in r.stderr
