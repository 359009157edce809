"""Pin the oracle (CPU restatement) against the reference's recorded answers
(tests/golden/survey_kat.json).  CPU only."""
import json
import os
import subprocess

import numpy as np
import pytest

from tests.wig import parse_table, write_contigs, write_wig

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "survey_kat.json")))


def run_case(tool, case, tmp_path):
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, case["contigs"])
    files = []
    for s in case["samples"]:
        p = tmp_path / f"{s['name']}.wig"
        write_wig(p, s["name"], s["fwd"], s["rev"])
        files.append(str(p))
    out = tmp_path / "out.txt"
    cmd = tool + ["-q", "-c", str(ct), "-o", str(out)] + case["args"] + files
    subprocess.run(cmd, check=True, capture_output=True)
    return parse_table(out)


@pytest.mark.parametrize("case", KAT["cases"], ids=lambda c: c["name"])
def test_survey_kat(orc_bin, case, tmp_path):
    _, col, rows = run_case([orc_bin, "regions"], case, tmp_path)
    got = [[r[0], int(r[1]), [int(x) for x in r[3:]]] for r in rows]
    assert got == case["expect"]


def test_kernel_edges_are_zero(oracle):
    bw = KAT["kernel_edges"]["bw"]
    for total in (1.0, 1 / 0.00925714, 216.0):
        k = oracle.kernel(bw, total)
        assert k[0] == 0.0 and k[-1] == 0.0
        assert np.all(k[1:-1] > 0)
        assert np.array_equal(k, k[::-1])


def test_q5_double_counted_coefficients(oracle):
    q = KAT["q5_countsum"]
    bw, bg = 5, 1.0
    k = oracle.kernel(bw, 1.0 / bg)
    prof = oracle.profile(bw, bg, 200, [100], np.array([q["counts"]], np.uint32),
                          coeffs=q["coeffs"])
    # centre cell holds k[bw] * countSum
    assert prof[99] == k[bw] * q["count_sum"]
