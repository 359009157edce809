"""CPU restatement of the reference's bin/convert_align -- TEST INFRASTRUCTURE
ONLY (parity checker for tests/test_gpu_convert.py; nothing in the product
imports it).  Pure Python, for small fixtures.

Follows, line by line in behaviour:
  src/convert_align.cpp:67-145            the driver (one parser across files,
                                          header lines, the self-check)
  misc/format.cpp:69-86                   BinomPosterior
  misc/format.cpp:103-128, 213-232        ParseAlignStream::open / printSummary
  misc/format.cpp:242-683                 parseAlign: BED, Eland multi, Corona,
                                          both wiggle formats, SAM, BAM
  misc/format.cpp:693-705                 readAlign's skip loop
  misc/data.cpp:301-314, 321-596          CountMap::add and its two iterators
  misc/format.cpp:1003-1089, 1164-1219    FormatOutStream's wiggle writer
  misc/bamtools/BamReader.cpp:621-700,
  misc/bamtools/BamAlignment.cpp:409-467  the BAM record fields it reads

Parity is unpinned against the reference binary (it needs Boost, absent
here): this is a restatement, checked against the behaviour
the reference source states.
"""
import math
import re
import struct
import sys
import zlib

M32 = 0xFFFFFFFF
BED_RE = re.compile(r"^[^\s]+\s\d+\s\d+\s[^\s]*\s[^\s]*?\s[+-]")
ELAND_RE = re.compile(r"^>.+?\t[ACGTN\.]+\t(\d+:\d+:\d+|RM|NM|QC)\t.+")
CORONA_RE = re.compile(r"^>\d+_\d+_\d+_F3")
SAM_HDR_RE = re.compile(r"^@[A-Za-z][A-Za-z](\t[A-Za-z][A-Za-z0-9]:[ -~]+)+$")
NAME1_RE = re.compile(r'name="(.+?)"')
NAME2_RE = re.compile(r"name=(.+?) ")
DIRNAME_RE = re.compile(r"(.+) ([+-])")
NM_RE = re.compile(r"^NM:i:(\d+)$")


class BadFormat(Exception):
    pass


class Exit(Exception):
    def __init__(self, code, msg=""):
        super().__init__(msg)
        self.code = code
        self.msg = msg


def lex_uint(s, maxv):
    """boost::lexical_cast<unsigned> (a leading '-' wraps)"""
    if not s:
        raise BadFormat
    neg = s[0] == "-"
    body = s[1:] if s[0] in "+-" else s
    if not body or not body.isdigit() or not body.isascii():
        raise BadFormat
    v = int(body)
    if v > maxv:
        raise BadFormat
    return (-v) & maxv if neg else v


def fname_prefix(p):
    p = p[p.rfind("/") + 1:]
    d = p.find(".")
    return p if d < 0 else p[:d]


def fmt17(v):
    return "%.17g" % v


class Binom:
    def __init__(self, L):
        c = 0.01 / (1 - 0.01)
        self.coef = [1.0] * (L + 1)
        for i in range(1, L + 1):
            self.coef[i] = self.coef[i - 1] * c * (L - i + 1) / i

    def prob(self, mm, hits):
        assert mm < len(self.coef) and len(hits) <= len(self.coef)
        den = 0.0
        for i, h in enumerate(hits):
            den += h * self.coef[i]
        assert den > 0
        return self.coef[mm] / den


def read_bam(path):
    """[(ref_name or None, pos, flag, mapq, l_seq, nm or None)] of a BAM file"""
    raw = open(path, "rb").read()
    data = bytearray()
    while raw:
        d = zlib.decompressobj(16 + 15)
        data += d.decompress(raw)
        raw = d.unused_data
    if data[:4] != b"BAM\1":
        return None
    p = 4
    l_text = struct.unpack_from("<I", data, p)[0]
    p += 4 + l_text
    n_ref = struct.unpack_from("<I", data, p)[0]
    p += 4
    refs = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<I", data, p)[0]
        refs.append(bytes(data[p + 4:p + 4 + ln - 1]).decode())
        p += 4 + ln + 4
    out = []
    while p + 4 <= len(data):
        bs = struct.unpack_from("<I", data, p)[0]
        r = p + 4
        rid, pos, bmn, fnc, l_seq = struct.unpack_from("<iiIIi", data, r)
        l_name, n_cig = bmn & 0xFF, fnc & 0xFFFF
        core = 32 + l_name + 4 * n_cig + (l_seq + 1) // 2 + l_seq
        tags = bytes(data[r + core:r + bs])
        nm = None
        q = 0
        while q + 3 <= len(tags):
            t, ty = tags[q:q + 2], chr(tags[q + 2])
            q += 3
            w = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}.get(ty)
            if t == b"NM":
                if ty in "cCsSiIA":
                    nm = int.from_bytes(tags[q:q + w], "little")
                break
            if w:
                q += w
            elif ty in "ZH":
                q = tags.index(b"\0", q) + 1
            else:
                break
        name = refs[rid] if 0 <= rid < len(refs) else ""
        out.append((name, pos, fnc >> 16, (bmn >> 8) & 0xFF, l_seq, nm))
        p += 4 + bs
    return out


class Parser:
    """ParseAlignStream as convert_align uses it (one object, reopened per file)"""

    def __init__(self, table, tol, use_len, offset, prob):
        self.names = [n for n, _ in table]
        self.lens = [L for _, L in table]
        self.index = {n: i for i, n in enumerate(self.names)}
        self.tol, self.use_len, self.offset = tol, use_len, offset
        self.read_len = use_len
        self.prob_thr = prob
        self.phred = 0 if prob == 0 else 255 if prob == 1 else -10 * math.log10(1 - prob)
        self.prob = Binom(use_len) if use_len else None
        self.line_no = 0
        self.err = []

    def idx(self, name):
        return self.index.get(name, len(self.names))

    def open(self, fname):
        self.fname = fname
        self.bam = fname.endswith(".bam")
        if self.bam:
            recs = read_bam(fname)
            self.bam_recs = iter(recs or [])
            self.bam_ok = recs is not None
        else:
            try:
                text = open(fname, "rb").read().decode("latin-1")
            except OSError:
                raise Exit(1, f"error: could not read {fname}\n\n")
            self.lines = text.split("\n")  # getline: count('\n') + 1 lines, the last may be empty
            self.li = 0
        self.format = 5 if self.bam else 0
        self.total = self.reject = self.oob = self.conf = 0
        self.name = fname_prefix(fname)
        self.a = dict(forward=True, contig=0, first=0, last=0, count=0, seq="")
        self.bam_done = not self.bam_ok if self.bam else False

    def good(self):
        return (not self.bam_done) if self.bam else self.li < len(self.lines)

    def read_line(self):
        if self.bam:
            return ""
        self.line_no += 1
        s = self.lines[self.li]
        self.li += 1
        return s

    def error(self, msg="bad format"):
        raise Exit(1, f"error: {msg} in {self.fname} line {self.line_no}\n\n")

    def read_align(self):
        nc = len(self.names)
        if self.good():
            self.parse(self.read_line())
        else:
            self.a["count"] = 0
            self.a["contig"] = nc
        while (self.a["count"] == 0 or self.a["contig"] == nc) and self.good():
            self.parse(self.read_line())
        return self.a

    def summary(self):
        s = (self.name + ": " if self.name else "") + f"{self.total} tags"
        if self.format in (2, 3, 4, 5):
            s += f"\n  {self.conf}" + (" confidently mapped" if self.prob_thr else " unique best")
            s += " hits (%.1f%%)" % (100 * self.conf / self.total if self.total else float("nan"))
            if self.prob_thr:
                s += f"\n  {self.reject} unique best hits rejected by filter (%.1f%%)" % (
                    100 * self.reject / self.total if self.total else float("nan"))
        if self.oob:
            s += f"\n{self.oob} out of contig bounds"
        return s + "\n"

    def parse(self, line):
        a = self.a
        nc = len(self.names)
        a["count"] = 0
        try:
            if (line == "" and self.format != 5) or line.startswith("#"):
                return
            if self.format == 0:
                if line.startswith("track"):
                    m = NAME1_RE.search(line) or NAME2_RE.search(line)
                    if m:
                        self.name = m.group(1)
                    if "type=wiggle_0" in line:
                        m2 = DIRNAME_RE.search(self.name)
                        if m2:
                            self.format = 6
                            self.name = m2.group(1)
                            a["forward"] = m2.group(2) == "+"
                        else:
                            self.format = 7
                            self.name = m.group(1) if m else ""
                            a["forward"] = True
                    else:
                        self.format = 1
                    return
                elif BED_RE.search(line):
                    self.format = 1
                elif ELAND_RE.search(line):
                    self.format = 2
                elif CORONA_RE.search(line):
                    self.format = 3
                elif SAM_HDR_RE.search(line):
                    self.format = 4
                else:
                    self.error()
            f = self.format
            if f == 1:
                if line.startswith("track"):
                    pass
                else:
                    fl = re.split(r"[\t ]", line)
                    if len(fl) < 6:
                        self.error()
                    st = fl[5][:1]
                    if st == "+":
                        a["forward"] = True
                    elif st == "-":
                        a["forward"] = False
                    else:
                        self.error()
                    a["contig"] = self.idx(fl[0])
                    a["seq"] = fl[3]
                    if a["forward"]:
                        a["first"] = (lex_uint(fl[1], M32) + 1) & M32
                        a["last"] = lex_uint(fl[2], M32)
                    else:
                        a["first"] = lex_uint(fl[2], M32)
                        a["last"] = (lex_uint(fl[1], M32) + 1) & M32
                    a["count"] = 1
                    self.total += 1
            elif f == 2:
                self.eland(line)
            elif f == 3:
                self.corona(line)
            elif f in (6, 7):
                if line[:1].isdigit():
                    if a["contig"] == nc:
                        return
                    d = max(line.rfind("\t"), line.rfind(" "))
                    if d < 0:
                        self.error()
                    a["first"] = lex_uint(line[:d], M32)
                    a["count"] = lex_uint(line[d + (2 if line[d + 1:d + 2] == "-" else 1):], M32)
                    u = self.use_len
                    if f == 6:
                        a["last"] = (a["first"] + (0 if u == 0 else (u - 1 if a["forward"] else -(u - 1)))) & M32
                    else:
                        a["last"] = (a["first"] + (0 if u == 0 else u - 1)) & M32
                    self.total += a["count"]
                elif re.match(r"^variableStep chrom=(.+)$", line):
                    a["contig"] = self.idx(line[19:])
                    return
                elif line.startswith("track") and NAME1_RE.search(line):
                    a["contig"] = nc
                    self.name = NAME1_RE.search(line).group(1)
                    if f == 6:
                        m2 = DIRNAME_RE.search(self.name)
                        if not m2:
                            self.error("strand not defined")
                        self.name = m2.group(1)
                        a["forward"] = m2.group(2) == "+"
                    return
                else:
                    self.error()
            elif f == 4:
                self.sam(line)
            elif f == 5:
                self.bam_rec()
            if a["count"] != 0 and a["contig"] != nc:
                if self.read_len:
                    a["last"] = (a["first"] + (self.read_len - 1 if a["forward"] else -(self.read_len - 1))) & M32
                o = self.offset
                if o:
                    first_i = a["first"] - (1 << 32) if a["first"] >= 1 << 31 else a["first"]
                    last_i = a["last"] - (1 << 32) if a["last"] >= 1 << 31 else a["last"]
                    if (a["forward"] and first_i > -o) or (not a["forward"] and last_i > o):
                        a["first"] = (a["first"] + (o if a["forward"] else -o)) & M32
                        a["last"] = (a["last"] + (o if a["forward"] else -o)) & M32
                    else:
                        self.oob += a["count"]
                        a["count"] = 0
                        return
                size = self.lens[a["contig"]]
                if a["first"] == 0 or a["first"] > size or a["last"] == 0 or a["last"] > size:
                    self.oob += a["count"]
                    a["count"] = 0
                    return
                self.conf += a["count"]
        except BadFormat:
            self.error()

    def eland(self, line):
        a = self.a
        fl = line.split("\t")
        if len(fl) < 4:
            self.error()
        self.total += 1
        if fl[3] == "-":
            return
        counts, best, found, unique = [], 0, False, False
        for t in [x for x in fl[2].split(":") if x]:
            counts.append(lex_uint(t, M32))
            if not found:
                if best > self.tol:
                    break
                if counts[-1] == 0:
                    best = (best + 1) & 0xFFFF
                else:
                    found = True
                    if counts[-1] == 1:
                        unique = True
                    else:
                        break
        if not unique:
            return
        a["seq"] = fl[1]
        use_seq = a["seq"]
        if self.use_len:
            if len(a["seq"]) >= self.use_len:
                use_seq = a["seq"][:self.use_len]
            else:
                self.error("sequence shorter than requested length")
        elif self.read_len:
            if len(use_seq) != self.read_len:
                self.error("different read length")
        else:
            self.read_len = len(a["seq"]) & 0xFFFF
            if self.prob_thr:
                self.prob = Binom(self.read_len)
        nN = use_seq.count("N")
        if self.prob and self.prob.prob(best, counts) < self.prob_thr:
            a["count"] = 0
            self.reject += 1
            return
        for hit in [x for x in fl[3].split(",") if x]:
            c = hit.find(":")
            if c >= 0:
                cs = hit[:c]
                sl = cs.find("/")
                a["contig"] = self.idx(fname_prefix(cs if sl < 0 else cs[sl + 1:]))
                hit = hit[c + 1:]
            d = min([k for k in (hit.find("F"), hit.find("R")) if k >= 0], default=-1)
            if d < 0:
                self.error()
            left = lex_uint(hit[:d], M32)
            a["forward"] = hit[d] == "F"
            hit = hit[d + 1:]
            mm, el = 0, 0
            w = min([k for k in (hit.find(ch) for ch in "ACGTN") if k >= 0], default=-1)
            if w < 0:
                v = lex_uint(hit, 0xFFFF)
                if v <= 2:
                    mm = v
            else:
                while w >= 0:
                    if w > 0:
                        el = (el + lex_uint(hit[:w], 0xFFFF)) & 0xFFFF
                    if el >= len(use_seq):
                        break
                    if hit[w] != "N":
                        mm = (mm + 1) & 0xFFFF
                    el = (el + 1) & 0xFFFF
                    hit = hit[w + 1:]
                    w = min([k for k in (hit.find(ch) for ch in "ACGTN") if k >= 0], default=-1)
                mm = (mm - nN) & 0xFFFF
            if mm == best:
                a["first"] = (left + (0 if a["forward"] else self.read_len - 1)) & M32
                if a["contig"] < len(self.names):
                    a["count"] = 1
                break

    def corona(self, line):
        a = self.a
        if not line.startswith(">"):
            return
        a["seq"] = self.read_line()
        self.total += 1
        at = line.find(",")
        if at < 0:
            return
        L = len(a["seq"]) - 1
        if self.use_len == 0:
            if self.read_len:
                if L != self.read_len:
                    self.error("different read length")
            else:
                self.read_len = L & 0xFFFF
                if self.prob_thr:
                    self.prob = Binom(self.read_len)
        elif L < self.use_len:
            self.error("sequence shorter than requested length")
        best = (self.tol + 1) & 0xFFFF
        mmc = [0]
        for h in line[at + 1:].split(","):
            f = h.split(".")
            if len(f) != 3:
                self.error()
            contig = self.idx(f[0])
            if contig >= len(self.names):
                break
            mm = lex_uint(f[2], 0xFFFF)
            if self.prob_thr:
                if len(mmc) >= ((mm + 1) & 0xFFFF):
                    mmc[mm] += 1
                else:
                    while len(mmc) < mm:
                        mmc.append(0)
                    mmc.append(1)
            if mm < best:
                a["contig"] = contig
                if not f[1].startswith("-"):
                    a["forward"] = True
                    a["first"] = (lex_uint(f[1], M32) + 1) & M32
                else:
                    a["forward"] = False
                    a["first"] = (lex_uint(f[1][1:], M32) + 1) & M32
                best = mm
                a["count"] = 1
            elif mm == best:
                a["count"] = 0
                if best == 0:
                    break
        if self.prob and a["count"] and self.prob.prob(best, mmc) < self.prob_thr:
            a["count"] = 0
            self.reject += 1

    def sam(self, line):
        a = self.a
        if line.startswith("@"):
            return
        fl = line.split("\t")
        if len(fl) < 10:
            self.error()
        flag = lex_uint(fl[1], 0xFFFF)
        if flag & 0x100:
            return
        self.total += 1
        if flag & (0x4 + 0x200):
            return
        if len(fl) > 11:
            ed = 0
            for x in fl:
                m = NM_RE.match(x)
                if m:
                    ed = lex_uint(m.group(1), 0x7FFFFFFF)
                    break
            if ed > self.tol:
                return
        if self.phred not in (0, 255) and lex_uint(fl[4], 0xFFFF) < self.phred:
            self.reject += 1
            return
        a["contig"] = self.idx(fl[2])
        if a["contig"] == len(self.names):
            return
        a["seq"] = fl[9]
        if self.use_len and len(a["seq"]) < self.use_len:
            self.error("sequence shorter than requested length")
        a["forward"] = not (flag & 0x10)
        a["first"] = (lex_uint(fl[3], M32) + (0 if a["forward"] else len(a["seq"]) - 1)) & M32
        ln = self.use_len if self.use_len else len(a["seq"])
        a["last"] = (a["first"] + (1 if a["forward"] else -1) * (ln - 1)) & M32
        a["count"] = 1

    def bam_rec(self):
        a = self.a
        r = next(self.bam_recs, None)
        if r is None:
            self.bam_done = True
            return
        name, pos, flag, mapq, l_seq, nm = r
        if flag & 0x100:
            return
        self.total += 1
        if (flag & 0x200) or (flag & 0x4):
            return
        if nm is not None and (nm - (1 << 32) if nm >= 1 << 31 else nm) > self.tol:
            return
        if self.phred not in (0, 255) and mapq < self.phred:
            self.reject += 1
            return
        a["contig"] = self.idx(name)
        if a["contig"] == len(self.names):
            return
        a["forward"] = not (flag & 0x10)
        a["first"] = (pos + (1 if a["forward"] else l_seq)) & M32
        ln = self.use_len if self.use_len else l_seq
        a["last"] = (a["first"] + (1 if a["forward"] else -1) * (ln - 1)) & M32
        a["count"] = 1


def convert_align(table, files, out_name, directional=True, tol=1, use_len=0, offset=0, prob=0.9,
                  assembly="", name="", quiet=True):
    """(exit code, output bytes or None, stderr text) of bin/convert_align"""
    err = []
    nc = len(table)
    counts = [dict() for _ in range(2 * nc)]  # [strand * nc + contig] -> {pos: count}
    tag_count = 0
    P = Parser(table, tol, use_len, offset, prob)
    try:
        for f in files:
            P.open(f)
            err.append(f"reading {f}...\n")
            if not quiet:
                err.append("0 tags read")
            while P.good():
                a = P.read_align()
                if a["count"] and a["contig"] < nc:
                    d = counts[(0 if a["forward"] else 1) * nc + a["contig"]]
                    d[a["first"]] = (d.get(a["first"], 0) + a["count"]) & M32
                    tag_count += a["count"]
            if not quiet:
                err.append("\r")
            err.append(P.summary())
    except Exit as e:
        err.append(e.msg)
        return e.code, None, "".join(err)
    err.append(f"{tag_count} usable tags\n")
    if tag_count == 0:
        err.append("error: nothing to do\n\n")
        return 1, None, "".join(err)
    track = name or fname_prefix(out_name)
    out = []
    for f in files:
        out.append(f"# original_file={f}\n")
    if prob != 0:
        out.append(f"# prob_threshold={fmt17(prob)}\n")
    out.append(f"# tags={tag_count}\n")

    def header(fwd):
        s = f'track name="{track}' + ((" +" if fwd else " -") if directional else "") + '"'
        if directional:
            s += ' description="' + (track if fwd else " ") + '"'
        s += " priority=3 visibility=full type=wiggle_0 alwaysZero=on color="
        s += ("0,0,255" if fwd else "255,0,0 altColor=255,0,0") if directional else "191,0,191"
        if assembly:
            s += " db=" + assembly
        return s + "\n"

    written = 0
    cur_contig, cur_fwd = None, None
    entries = []
    if directional:
        for st in (0, 1):
            for c in range(nc):
                for p in sorted(counts[st * nc + c]):
                    entries.append((st == 0, c, p, counts[st * nc + c][p]))
    else:
        for c in range(nc):
            fw, rv = counts[c], counts[nc + c]
            for p in sorted(set(fw) | set(rv)):
                entries.append((True, c, p, (fw.get(p, 0) + rv.get(p, 0)) & M32))
    for fwd, c, p, k in entries:
        if k == 0:
            continue
        if directional:
            if cur_contig is None or cur_fwd != fwd:
                cur_fwd = fwd
                cur_contig = None
                out.append(header(fwd))
        elif cur_contig is None:
            out.append(header(True))
        if cur_contig != c:
            cur_contig = c
            out.append(f"variableStep chrom={table[c][0]}\n")
        out.append(f"{p} " + ("" if (fwd or not directional) else "-") + f"{k}\n")
        written += k
    if written != tag_count:
        err.append(f"error: {written} {tag_count}\n")
        return 1, "".join(out).encode("latin-1"), "".join(err)
    return 0, "".join(out).encode("latin-1"), "".join(err)


if __name__ == "__main__":
    sys.exit("test infrastructure: import convert_align() from tests")
