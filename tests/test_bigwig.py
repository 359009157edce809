"""bin/wigs2bigwigs (the native replacement of extras/wigs2bigwigs.pl +
UCSC wigToBigWig -clip): the bigWig files are decoded with
an independent reader of the BBI layout (header, chromosome B+ tree, R-tree
index, zlib sections) and must hold exactly the intervals and float32 values
of the wiggle input (clipped at the chromosome ends), and the printed track
headers must be the script's.  Host-only: runs on CPU.

Zoom levels are checked against a restatement of wigToBigWig's summary
algorithm (bbiAddRangeToSummary: bins that start at a run's first item,
items split across bin edges, sums in double stored as float).

Parity note: wigToBigWig is not in this image, so the files are checked for
content, not bytes (its section sizes and its choice of levels are its own)."""
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
    # zoom levels: headers after the 64-byte header, records through each R-tree
    zl = []
    for z in range(zooms):
        red, _, zdata, zindex = struct.unpack_from("<IIQQ", b, 64 + 24 * z)
        zm, zbs, zitems = struct.unpack_from("<IIQ", b, zindex)
        assert zm == 0x2468ACE0
        count, = struct.unpack_from("<I", b, zdata)
        zblocks = []

        def walk_z(off):
            leaf, _, cnt = struct.unpack_from("<BBH", b, off)
            off += 4
            for _ in range(cnt):
                if leaf:
                    zblocks.append(struct.unpack_from("<IIIIQQ", b, off))
                    off += 32
                else:
                    walk_z(struct.unpack_from("<IIIIQ", b, off)[4])
                    off += 24
        walk_z(zindex + 48)
        recs = []
        for c0, s0, c1, s1, doff, dsize in zblocks:
            raw = zlib.decompress(b[doff:doff + dsize])
            assert len(raw) <= ubuf and len(raw) % 32 == 0
            for k in range(len(raw) // 32):
                r = struct.unpack_from("<IIIIffff", raw, 32 * k)
                assert r[0] == c0 == c1 and s0 <= r[1] and r[2] <= s1
                recs.append(r)
        assert len(recs) == count
        zl.append((red, recs))
    return out, chroms, zl


def summarise(items_by_cid, csize, red):
    """wigToBigWig's zoom records (bbiAddRangeToSummary), restated"""
    out = []
    for cid in sorted(items_by_cid):
        cur = None
        for s, e, v in items_by_cid[cid]:
            e = min(e, csize[cid])
            while s < e:
                if cur is None or cur[2] <= s:
                    st = s if (cur is None or cur[2] + red <= s) else cur[2]
                    cur = [cid, st, min(st + red, csize[cid]), 0, v, v, 0.0, 0.0]
                    out.append(cur)
                ov = min(e, cur[2]) - max(s, cur[1])
                cur[3] += ov
                cur[4] = min(cur[4], v)
                cur[5] = max(cur[5], v)
                cur[6] += v * ov
                cur[7] += v * v * ov
                s += ov
    return out


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
        got, chroms, zl = read_bigwig(tmp_path / f"p{strand}.bw")
        assert {v[0]: v[1] for v in chroms.values()} == {c: sizes[c] for c in items}
        assert set(got) == set(items)
        for c in items:
            assert got[c] == items[c], c
        # zoom levels: 10x the average item span, then 4x per level, each
        # with fewer records than the one before; every record as restated
        cid = {name: i for i, (name, _) in chroms.items()}
        by_cid = {cid[c]: v for c, v in items.items()}
        csize = {i: L for i, (_, L) in chroms.items()}
        n = sum(len(v) for v in items.values())
        span = sum(e - s for v in items.values() for s, e, _ in v)
        assert len(zl) >= 3
        assert zl[0][0] == max(1, (span + n // 2) // n) * 10
        prev = n
        for k, (red, recs) in enumerate(zl):
            if k:
                assert red == 4 * zl[k - 1][0]
            ref = summarise(by_cid, csize, red)
            assert len(recs) == len(ref) < prev
            prev = len(recs)
            for r, q in zip(recs, ref):
                assert r[:4] == tuple(q[:4]) and r[4] == q[4] and r[5] == q[5]
                assert r[6] == np.float32(q[6]) and r[7] == np.float32(q[7])
            assert sum(r[3] for r in recs) == span


def test_wigs2bigwigs_errors(tmp_path):
    (tmp_path / "s.sizes").write_text("chr1\t1000\n")
    (tmp_path / "a.wig").write_text("variableStep chrom=chr1\n5 1\n")
    r = subprocess.run([BIN, "--sizes", "s.sizes", "a.wig"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode != 0 and "error: no track defined at line 1" in r.stderr
    (tmp_path / "b.wig").write_text('track name="b" type=wiggle_0\nvariableStep chrom=chrQ\n5 1\n')
    r = subprocess.run([BIN, "--sizes", "s.sizes", "b.wig"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode != 0 and "chrQ" in r.stderr
