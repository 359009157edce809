"""Writers for small wiggle/contig-table fixtures (the formats of
misc/format.cpp:1043-1075, 1164-1219 as written by bin/convert_align)."""


def write_contigs(path, contigs):
    with open(path, "w") as f:
        for name, size in contigs:
            f.write(f"{name}\t{size}\n")


def write_wig(path, name, fwd, rev, tags=None, header=True):
    """fwd/rev: {contig: [(pos, count), ...]} in the order to write."""
    total = sum(c for d in (fwd, rev) for v in d.values() for _, c in v)
    with open(path, "w") as f:
        f.write("# original_file=synthetic\n")
        if header:
            f.write(f"# tags={total if tags is None else tags}\n")
        f.write(f'track name="{name} +" description="{name}" priority=3 visibility=full '
                'type=wiggle_0 alwaysZero=on color=0,0,255\n')
        for c, v in fwd.items():
            f.write(f"variableStep chrom={c}\n")
            for p, k in v:
                f.write(f"{p} {k}\n")
        f.write(f'track name="{name} -" description=" " priority=3 visibility=full '
                'type=wiggle_0 alwaysZero=on color=255,0,0 altColor=255,0,0\n')
        for c, v in rev.items():
            f.write(f"variableStep chrom={c}\n")
            for p, k in v:
                f.write(f"{p} -{k}\n")
    return total


def parse_table(path):
    """(header lines, column line, rows as lists of fields)"""
    hdr, col, rows = [], None, []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if col is None and (not line or line.startswith("#")):
                hdr.append(line)
            elif col is None:
                col = line
            else:
                rows.append(line.split("\t"))
    return hdr, col, rows
