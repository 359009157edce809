"""tags_in_regions on the GPU (src/tags_in_regions.cpp:131-199).

* up_tir_query against a plain-Python restatement of the reference's skip and
  count loops started at the stream's first record, on sorted directional
  streams, position-merged (nondirectional) streams, streams whose contig
  order differs from the table's, and shuffled streams (many unsorted runs:
  the device hands those pairs to the host, UP_TIR_HOST);
* bin/tags_in_regions byte-identical to the oracle CLI, including the cursor
  cases the device answer cannot take (regions out of order, forward regions
  after reverse ones on a one-contig table, quirk Q12) and input errors that
  the reference meets -- or never reaches -- part-way through a stream."""
import os
import subprocess

import numpy as np
import pytest

from tests.test_cli import BIN, HG_LIKE, compare_tool, make_inputs, run
from tests.wig import write_contigs, write_wig

TIR_HOST = 0xFFFFFFFF


def walk_from_start(key, cnt, fwd, c, left, right, f):
    """the reference's loops (tags_in_regions.cpp:185-190) from record 0"""
    n = len(key)
    kl, kr = (c << 32) | left, (c << 32) | right
    s = 0
    while s < n and not (fwd[s] == f and key[s] >= kl):
        s += 1
    e, h = s, 0
    while e < n and (key[e] >> 32) == c and key[e] <= kr:
        h = (h + int(cnt[e])) & 0xFFFFFFFF
        e += 1
    return s, e, h


def make_stream(rng, n_contigs, per_contig, mode):
    """(contig, first, count, forward) arrays in stream order"""
    recs = []
    for strand in (True, False):
        for c in range(n_contigs):
            pos = np.unique(rng.integers(1, 200_000, per_contig))
            for p in pos:
                recs.append((c, int(p), int(rng.integers(1, 6)) if rng.random() > 0.01
                             else int(rng.integers(1, 1 << 31)), strand))
    if mode == "nondir":    # both strands merged by position
        recs.sort(key=lambda r: (r[0], r[1], not r[3]))
    elif mode == "order":   # wiggle contig order differs from the table's
        perm = rng.permutation(n_contigs)
        recs.sort(key=lambda r: (not r[3], int(np.where(perm == r[0])[0][0]), r[1]))
    elif mode == "shuffled":
        idx = rng.permutation(len(recs))
        recs = [recs[i] for i in idx]
    a = np.array([(r[0], r[1], r[2], r[3]) for r in recs], dtype=np.int64)
    return a[:, 0].astype(np.uint32), a[:, 1].astype(np.uint32), a[:, 2].astype(np.uint32), \
        a[:, 3].astype(np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["dir", "nondir", "order", "shuffled", "empty"])
def test_tir_query_matches_walk(gpu_lib, mode):
    rng = np.random.default_rng({"dir": 1, "nondir": 2, "order": 3, "shuffled": 4, "empty": 5}[mode])
    nc = 5
    streams = []
    for s in range(3):
        if mode == "empty" and s == 1:
            z = np.zeros(0, np.uint32)
            streams.append((z, z, z, z.astype(np.uint8)))
        else:
            streams.append(make_stream(rng, nc, 300 if mode == "shuffled" else 3000,
                                       "dir" if mode == "empty" else mode))
    R = 700
    rc = rng.integers(0, nc + 1, R).astype(np.uint32)  # contig nc: not in any stream
    rl = rng.integers(0, 200_000, R).astype(np.uint32)
    rr = (rl + rng.integers(0, 3000, R)).astype(np.uint32)
    rf = rng.integers(0, 2, R).astype(np.uint8)
    rr[:5] = 0xFFFFFFFF  # right edge at the uint32 maximum (wrapped -e)
    with gpu_lib.Tir(0) as t:
        for i, (c, p, k, f) in enumerate(streams):
            t.set_stream(i, c, p, k, f)
        first, end, hits = t.query(rc, rl, rr, rf)
    host = 0
    for i, (c, p, k, f) in enumerate(streams):
        key = (c.astype(np.uint64) << np.uint64(32)) | p.astype(np.uint64)
        key = [int(x) for x in key]
        for r in range(R):
            if first[r, i] == TIR_HOST:
                assert mode == "shuffled"
                host += 1
                continue
            want = walk_from_start(key, k, f, int(rc[r]), int(rl[r]), int(rr[r]), int(rf[r]))
            assert (first[r, i], end[r, i], hits[r, i]) == want, (mode, i, r)
    if mode == "shuffled":
        assert host > 0  # the unsorted stream's long walks went to the host


@pytest.mark.gpu
def test_tir_prefix_tables_large(gpu_lib):
    """a 3-million-record stream (several scan blocks of the table build, the
    block-carry kernel's chunk loop) and the uint32 wrap of the hit sum"""
    rng = np.random.default_rng(9)
    n = 3_000_001
    c = np.sort(rng.integers(0, 4, n)).astype(np.uint32)
    p = np.zeros(n, np.uint32)
    for k in range(4):
        m = c == k
        p[m] = np.sort(rng.choice(2_000_000_000, int(m.sum()), replace=False))
    k = rng.integers(1, 1 << 20, n).astype(np.uint32)
    k[::1000] = 0xFFFFFFF0
    f = (rng.random(n) < 0.5).astype(np.uint8)
    R = 4000
    rc = rng.integers(0, 4, R).astype(np.uint32)
    rl = rng.integers(0, 2_000_000_000, R).astype(np.uint32)
    rr = (rl.astype(np.uint64) + rng.integers(0, 50_000_000, R)).clip(0, 0xFFFFFFFF).astype(np.uint32)
    rf = rng.integers(0, 2, R).astype(np.uint8)
    with gpu_lib.Tir(0) as t:
        t.set_stream(0, c, p, k, f)
        first, end, hits = t.query(rc, rl, rr, rf)
    key = (c.astype(np.uint64) << np.uint64(32)) | p.astype(np.uint64)
    csum = np.concatenate([[0], np.cumsum(k, dtype=np.uint64)])
    nextf = np.full(n + 1, n, np.int64)
    nextr = np.full(n + 1, n, np.int64)
    for arr, want in ((nextf, 1), (nextr, 0)):
        idx = np.where(f == want)[0]
        pos = np.searchsorted(idx, np.arange(n + 1))
        arr[:] = np.where(pos < len(idx), idx[np.minimum(pos, len(idx) - 1)], n)
    for r in range(R):
        kl = (int(rc[r]) << 32) | int(rl[r])
        kr = (int(rc[r]) << 32) | int(rr[r])
        j = int(np.searchsorted(key, np.uint64(kl), "left"))
        s = int((nextf if rf[r] else nextr)[j])
        e = s
        if s < n and key[s] <= kr and (int(key[s]) >> 32) == rc[r]:
            e = int(np.searchsorted(key, np.uint64(kr), "right"))
        h = int(csum[e] - csum[s]) & 0xFFFFFFFF
        assert (first[r, 0], end[r, 0], hits[r, 0]) == (s, e, h), r


# ---- bin/tags_in_regions vs the oracle CLI ----

@pytest.mark.gpu
def test_tags_in_regions_cli_matches_oracle(orc_bin, gpu_lib, tmp_path):
    """build a region table with the oracle, then count 2 extra samples"""
    ct, files = make_inputs(tmp_path, 5, HG_LIKE, 3)
    regions = tmp_path / "regions.txt"
    run([orc_bin, "regions", "-q", "-f", "-c", ct, "-o", str(regions), files[0]], tmp_path)
    for extra in (["-e", "30"], [], ["-s", "25"], ["-s", "40,-12"], ["-e", "4294967295"]):
        compare_tool(orc_bin, tmp_path, "tags_in_regions",
                     ["-c", ct, "-f", str(regions)] + extra + files[1:])
    # nondirectional input table
    nd = tmp_path / "nd.txt"
    run([orc_bin, "regions", "-q", "-D", "-c", ct, "-o", str(nd), files[0]], tmp_path)
    compare_tool(orc_bin, tmp_path, "tags_in_regions", ["-D", "-c", ct, "-f", str(nd)] + files[1:],
                 outname="nd_out.txt")


@pytest.mark.gpu
def test_tags_in_regions_q12_reverse_mislabel(orc_bin, gpu_lib, tmp_path):
    """Q12: a forward-labelled reverse region counts 0 (no strand check in the
    count loop; survey probe `chrA:5011-5162 55 0`)."""
    write_contigs(tmp_path / "ct.txt", [("chrA", 20000)])
    write_wig(tmp_path / "a.wig", "a", {}, {"chrA": [(5100, 30), (8000, 30)]})
    (tmp_path / "r.txt").write_text("# x\n\tkurtosis\ta\nchrA:5011-5162\t1.00\t30\n"
                                    "chrA:8060-7940\t1.00\t30\n")
    out = compare_tool(orc_bin, tmp_path, "tags_in_regions",
                       ["-c", "ct.txt", "-f", "r.txt", "a.wig"])
    rows = [l.split("\t") for l in out.strip().split("\n") if not l.startswith(("#", "\t"))]
    # the forward-labelled region skips (and so consumes) the reverse tags
    assert rows[0][-1] == "0" and rows[1][-1] == "0"


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_tags_in_regions_cursor_cases(orc_bin, gpu_lib, tmp_path, seed):
    """region rows the device answer cannot take: a one-contig table (forward
    and reverse regions interleave, quirk Q4, so forward regions come after
    the cursor entered the reverse track), rows shuffled out of order,
    overlapping extended rows, and a wiggle whose contig order differs from
    the table's"""
    rng = np.random.default_rng(seed)
    one = [("chrA", 120_000)]
    ct, files = make_inputs(tmp_path, seed, one, 3)
    regions = tmp_path / "regions.txt"
    run([orc_bin, "regions", "-q", "-c", ct, "-o", str(regions), files[0]], tmp_path)
    text = regions.read_text().split("\n")
    assert any("-" in l and l.startswith("chrA:") for l in text)
    compare_tool(orc_bin, tmp_path, "tags_in_regions", ["-c", ct, "-f", str(regions)] + files[1:])
    compare_tool(orc_bin, tmp_path, "tags_in_regions",
                 ["-c", ct, "-f", str(regions), "-e", "3000"] + files[1:], outname="ext.txt")
    hdr = [l for l in text if l.startswith("#") or l.startswith("\t")]
    rows = [l for l in text if l and not l.startswith(("#", "\t"))]
    shuf = tmp_path / "shuffled.txt"
    shuf.write_text("\n".join(hdr + [rows[i] for i in rng.permutation(len(rows))]) + "\n")
    compare_tool(orc_bin, tmp_path, "tags_in_regions", ["-c", ct, "-f", str(shuf)] + files[1:],
                 outname="shuf.txt")
    # contig order: the table lists chrC first, the wiggles chrA first
    d2 = tmp_path / "order"
    d2.mkdir()
    ct2, files2 = make_inputs(d2, seed + 100, HG_LIKE, 2)
    rev_ct = tmp_path / "rev_contigs.txt"
    write_contigs(rev_ct, list(reversed(HG_LIKE)))
    reg2 = tmp_path / "regions2.txt"
    run([orc_bin, "regions", "-q", "-c", str(rev_ct), "-o", str(reg2), files2[0]], tmp_path)
    compare_tool(orc_bin, tmp_path, "tags_in_regions", ["-c", str(rev_ct), "-f", str(reg2), files2[1]],
                 outname="order.txt")


def _both(orc_bin, tmp_path, args):
    a = subprocess.run([orc_bin, "tags_in_regions"] + args + ["-o", str(tmp_path / "ra.txt")],
                       cwd=tmp_path, capture_output=True, text=True)
    b = subprocess.run([os.path.join(BIN, "tags_in_regions")] + args + ["-o", str(tmp_path / "rb.txt")],
                       cwd=tmp_path, capture_output=True, text=True)
    return a, b


@pytest.mark.gpu
def test_tags_in_regions_input_errors(orc_bin, gpu_lib, tmp_path):
    """an unreadable wiggle line is reported only if a cursor reaches it (the
    reference reads lazily); a malformed region row after the rows the
    cursors walk is reported after them"""
    write_contigs(tmp_path / "ct.txt", [("chrA", 50000)])
    good = "".join(f"{p} 2\n" for p in range(1000, 3000, 50))
    for late in (True, False):
        body = ('# tags=100\ntrack name="a +" description="a" type=wiggle_0\nvariableStep chrom=chrA\n'
                + good + ("40000 3\nbogus line\n" if late else "bogus line\n40000 3\n"))
        (tmp_path / "a.wig").write_text(body)
        (tmp_path / "r.txt").write_text("#h\n\tx\nchrA:1100-1500\t1\nchrA:2000-2990\t1\n")
        a, b = _both(orc_bin, tmp_path, ["-c", "ct.txt", "-f", "r.txt", "a.wig"])
        assert (a.returncode, b.returncode) == ((0, 0) if late else (1, 1)), (a.stderr, b.stderr)
        if late:
            assert (tmp_path / "ra.txt").read_bytes() == (tmp_path / "rb.txt").read_bytes()
        else:
            assert a.stderr.strip().split("\n")[-1] == b.stderr.strip().split("\n")[-1]
    # a bad region row: the stream error before it (row 2 reaches "bogus") wins
    (tmp_path / "r.txt").write_text("#h\n\tx\nchrA:1100-1500\t1\nchrA:2900-45000\t1\nnot a row\n")
    a, b = _both(orc_bin, tmp_path, ["-c", "ct.txt", "-f", "r.txt", "a.wig"])
    assert a.returncode == b.returncode == 1
    assert a.stderr.strip().split("\n")[-1] == b.stderr.strip().split("\n")[-1]
    (tmp_path / "a.wig").write_text('# tags=10\ntrack name="a +" description="a" type=wiggle_0\n'
                                    "variableStep chrom=chrA\n" + good)
    a, b = _both(orc_bin, tmp_path, ["-c", "ct.txt", "-f", "r.txt", "a.wig"])
    assert a.returncode == b.returncode == 1
    assert a.stderr.strip().split("\n")[-1] == b.stderr.strip().split("\n")[-1]


def test_tags_in_regions_fails_loudly_without_gpu(tmp_path):
    """CPU container: the GPU path has no CPU fallback"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    write_contigs(tmp_path / "ct.txt", [("chrA", 20000)])
    write_wig(tmp_path / "a.wig", "a", {"chrA": [(5100, 30)]}, {})
    (tmp_path / "r.txt").write_text("# x\n\tk\nchrA:5011-5162\t1\n")
    r = subprocess.run([os.path.join(BIN, "tags_in_regions"), "-c", "ct.txt", "-f", "r.txt", "-o",
                        "o.txt", "a.wig"], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 1 and "no HIP device" in r.stderr
