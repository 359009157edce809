"""C-ABI boundary checks that need no GPU: the library loads, exports every
entry point include/unipeak_hip.h declares, and its host-side Kernel
restatement matches the oracle bit for bit."""
import ctypes
import os
import re

import numpy as np
import pytest

from unipeak_amd import capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "unipeak_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(up_[a-z_]+)\s*\(", src)))


def test_header_constants_match_capi():
    """the Python mirror's copies of header constants"""
    src = open(os.path.join(ROOT, "include", "unipeak_hip.h")).read()
    m = re.search(r"#define\s+UP_MAX_IN_FLIGHT\s+(\d+)", src)
    assert m and int(m.group(1)) == capi.MAX_IN_FLIGHT


def test_header_bw_limit_matches_kernels():
    """the boundary's stated parallel-scan limit is the kernels' kMaxBw, and
    every bandwidth the header, INTEGRATION.md and DESIGN.md name as the
    replay threshold is that value (rounds 3 and 4 left stale copies)"""
    hdr = open(os.path.join(ROOT, "include", "unipeak_hip.h")).read()
    ker = open(os.path.join(ROOT, "unipeak_amd", "csrc", "kernels.h")).read()
    m = re.search(r"#define\s+UP_MAX_PARALLEL_BW\s+(\d+)", hdr)
    k = re.search(r"constexpr int kMaxBw = (\d+);", ker)
    assert m and k and int(m.group(1)) == int(k.group(1))
    lim = int(k.group(1))
    for f in ("include/unipeak_hip.h", "INTEGRATION.md", "DESIGN.md"):
        txt = open(os.path.join(ROOT, f)).read()
        for v in re.findall(r"(?:bw|-b)\s*(?:>|&gt;)\s*(\d+)", txt):
            assert int(v) in (lim, 63), (f, v)  # 63: the NH=1 kernel's own width


def test_library_exports_header():
    L = capi.load_library()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(capi.EXPORTS)


def test_version_and_errors():
    L = capi.load_library()
    assert L.up_version() == 10000
    assert L.up_strerror(-5) == b"configuration outside the GPU path"


@pytest.mark.parametrize("bw", [1, 5, 50, 63, 64, 100, 127, 500])
@pytest.mark.parametrize("total", [1.0, 1 / 0.00925714, 1 / 0.0029253, 341.25])
def test_kernel_weights_match_oracle(oracle, bw, total):
    a = capi.kernel_weights(bw, total)
    b = oracle.kernel(bw, total)
    assert a.tobytes() == b.tobytes()


def test_open_without_device_fails_cleanly():
    if capi.device_count() > 0:
        pytest.skip("device present")
    L = capi.load_library()
    ctx = ctypes.c_void_p()
    assert L.up_open(0, ctypes.byref(ctx)) == -6
