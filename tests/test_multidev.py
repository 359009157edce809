"""The CLIs' multi-device path (units LPT-spread over the visible GPUs, quirk-Q1
leak chains kept on one device, candidates merged back into the reference's
emission order; tags_in_regions: samples dealt round-robin) -- exercised on a
one-GPU box through UNIPEAK_SHARE_DEVICE=N: N logical devices, each its own
context, all on HIP device 0.  Every output byte-identical to the oracle CLI,
as with one device."""
import os
import zlib

import numpy as np
import pytest

from tests.test_cli import (HG_LIKE, Q1_CASES, compare_tool, gen_head_sample, make_inputs, run)
from tests.wig import write_contigs, write_wig

pytestmark = pytest.mark.gpu

MANY = [(f"chr{i}", 20_000 + 7_000 * (i % 5)) for i in range(12)]


@pytest.fixture
def share(monkeypatch):
    def set_n(n):
        monkeypatch.setenv("UNIPEAK_SHARE_DEVICE", str(n))
    return set_n


@pytest.mark.parametrize("ndev", [2, 3, 7])
@pytest.mark.parametrize("case", [
    ("directional", MANY, 1, ["-f"], {}),
    ("controls_coeffs", MANY, 3, ["-f", "-e", "3", "-z", "p"], {}),
    ("nondir_corr", MANY, 2, ["-D", "-y", "-f", "-s", "60"], {"shift_rev": 120}),
    ("replay_r0", HG_LIKE, 1, ["-f", "-r", "0"], {}),
], ids=lambda c: c[0] if isinstance(c, tuple) else str(c))
def test_regions_multi_device(orc_bin, gpu_lib, tmp_path, share, ndev, case):
    share(ndev)
    name, contigs, ns, args, kw = case
    ct, files = make_inputs(tmp_path, zlib.crc32(name.encode()) % 10_000, contigs, ns, **kw)
    out = compare_tool(orc_bin, tmp_path, "regions", ["-q", "-c", ct] + args + files)
    assert out.count("\n") > 10


@pytest.mark.parametrize("case", [c for c in Q1_CASES if c[4]], ids=lambda c: c[0])
def test_regions_multi_device_q1_chains(orc_bin, gpu_lib, tmp_path, share, case):
    """leak chains (a unit whose adds all sit at <= bw) must stay on one device"""
    share(4)
    name, bw, ns, args, tiny = case
    rng = np.random.default_rng(zlib.crc32((name + "md").encode()))
    contigs = [("c0", 9000), ("c1", 4000), ("c2", 400), ("c3", 7000), ("c4", 5000)]
    ct = tmp_path / "contigs.txt"
    write_contigs(ct, contigs)
    files = []
    for i in range(ns):
        fwd, rev = gen_head_sample(rng, contigs, bw, tiny)
        p = tmp_path / f"s{i}.wig"
        write_wig(p, f"s{i}", fwd, rev)
        files.append(str(p))
    compare_tool(orc_bin, tmp_path, "regions", ["-q", "-c", str(ct), "-b", str(bw), "-m", "3000"] + args + files)


def test_strand_shift_and_tags_in_regions_multi_device(orc_bin, gpu_lib, tmp_path, share):
    share(3)
    ct, files = make_inputs(tmp_path, 77, MANY, 4, shift_rev=150)
    rep = compare_tool(orc_bin, tmp_path, "strand_shift", ["-x", "100", "-c", ct, files[0]], "shift.txt")
    assert "# best_shift=" in rep
    run([orc_bin, "regions", "-q", "-f", "-c", ct, "-o", "regs.txt", files[0]], tmp_path)
    compare_tool(orc_bin, tmp_path, "tags_in_regions", ["-c", ct, "-f", "regs.txt"] + files[1:], "tir.txt")


def test_share_knob_is_multi_device(gpu_lib, tmp_path, share):
    """the knob really splits the run: -q off, the CLI reports one pass per
    logical device (UNIPEAK_TIMING lines name each device's up_run)"""
    share(3)
    ct, files = make_inputs(tmp_path, 5, MANY, 1)
    env = dict(os.environ, UNIPEAK_TIMING="1")
    import subprocess
    r = subprocess.run([os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin",
                        "regions"), "-c", ct, "-o", "o.txt"] + files, cwd=tmp_path, capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stderr[-1000:]
    assert r.stderr.count("gpu: up_run") == 3, r.stderr[-3000:]
