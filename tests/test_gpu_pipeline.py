"""Pipelined passes (up_run_async / up_run_wait, include/unipeak_hip.h):
two, three or UP_MAX_IN_FLIGHT passes in flight (each on its own stream and buffers, a pass's
K1a overlapping the previous passes' K1b/K2/K3), each delivering into the
record target that was set when it was launched, give exactly the records of
the blocking up_run; one launch more than UP_MAX_IN_FLIGHT is refused; state
cannot change under a pass in flight; the K2 segmentation (two launches,
re-armed counters) stays exact across many passes and across units whose
strip counts span several K2 blocks."""
import ctypes

import numpy as np
import pytest

from tests.gen import random_unit

pytestmark = pytest.mark.gpu

UP_E_STATE = -4


def _load(g, rng, lengths, bw):
    for L in lengths:
        u = g.add_unit(L)
        pos, cnt = random_unit(rng, L, bw)
        g.scatter(u, 0, 0, pos, cnt[:, 0])


def _target(cap, S, rec):
    nbytes = 8 + cap * (rec + 4 * S)
    buf = np.zeros(nbytes + 4096, np.uint8)
    off = (-buf.ctypes.data) % 4096
    return buf, off


def _parse(buf, off, cap, S, dtype):
    raw = buf[off:]
    n = int(raw[:8].view(np.uint64)[0])
    recs = raw[8:8 + n * dtype.itemsize].view(dtype).copy()
    c0 = 8 + cap * dtype.itemsize
    cnt = raw[c0:c0 + n * S * 4].view(np.uint32).reshape(n, S).copy()
    return recs, cnt


@pytest.mark.parametrize("seed,depth", [(0, 2), (1, 2), (2, 3), (3, 3), (4, 5)])
def test_async_matches_blocking(gpu_lib, seed, depth):
    capi = gpu_lib
    rng = np.random.default_rng(seed)
    bw = 50
    lengths = [int(x) for x in rng.integers(30_000, 2_500_000, size=7)]
    with capi.Lib(0) as g:
        g.set_params(bw, 1, 0.003)
        _load(g, rng, lengths, bw)
        n = g.run()
        ref, rcnt = g.regions(n)
        assert n > 0
        cap = n + 16
        bufs = [_target(cap, 1, capi.REGION_DTYPE.itemsize) for _ in range(depth)]
        for b, off in bufs:
            g.host_register(b[off:].ctypes.data, len(b) - off)
        for timing in (0, 1, 2):
            g.set_timing(timing)
            got = []
            npass = 7
            for i in range(npass):
                b, off = bufs[i % depth]
                g.set_record_target(b[off:].ctypes.data, cap)
                g.run_async()
                if i >= depth - 1:
                    m = g.run_wait()
                    pb, poff = bufs[(i - depth + 1) % depth]
                    got.append((m,) + _parse(pb, poff, cap, 1, capi.REGION_DTYPE))
                # state is frozen while passes are in flight
                with pytest.raises(capi.UpError) as e:
                    g.set_params(bw, 1, 0.003)
                assert e.value.code == UP_E_STATE
            for j in range(npass - depth + 1, npass):
                m = g.run_wait()
                b, off = bufs[j % depth]
                got.append((m,) + _parse(b, off, cap, 1, capi.REGION_DTYPE))
            with pytest.raises(capi.UpError):
                g.run_wait()  # nothing in flight
            assert len(got) == npass
            for m, recs, cnt in got:
                assert m == n
                assert recs.tobytes() == ref.tobytes()
                assert np.array_equal(cnt, rcnt)
        g.set_record_target(0, 0)
        g.set_timing(2)
        assert g.run() == n


def test_async_host_delivery_and_growth(gpu_lib):
    """host delivery (no target), first pass grows the record areas while
    later passes are in flight; one pass more than UP_MAX_IN_FLIGHT is refused"""
    capi = gpu_lib
    rng = np.random.default_rng(5)
    bw = 5  # narrow windows: most tags are regions of their own
    with capi.Lib(0) as g:
        g.set_params(bw, 1, 0.0005)  # low background: every tag opens a region
        for L in (3_000_000, 1_200_000):
            u = g.add_unit(L)
            pos, cnt = random_unit(rng, L, bw, n_bg=L // 25)
            g.scatter(u, 0, 0, pos, cnt[:, 0])
        for _ in range(capi.MAX_IN_FLIGHT):
            g.run_async()
        with pytest.raises(capi.UpError) as e:
            g.run_async()
        assert e.value.code == UP_E_STATE
        n1 = g.run_wait()
        r1, c1 = g.regions(n1)
        n2 = g.run_wait()
        r2, c2 = g.regions(n2)
        for _ in range(capi.MAX_IN_FLIGHT - 3):
            g.run_wait()
        n4 = g.run_wait()
        r4, c4 = g.regions(n4)
        n3 = g.run()
        r3, c3 = g.regions(n3)
    assert n1 == n2 == n3 == n4 and n1 > (1 << 16)  # beyond the initial record capacity
    assert r1.tobytes() == r2.tobytes() == r3.tobytes() == r4.tobytes()
    assert np.array_equal(c1, c3) and np.array_equal(c2, c3) and np.array_equal(c4, c3)


def test_many_units_many_blocks(gpu_lib, oracle):
    """strip counts spanning several 256-strip K2 blocks; every unit checked
    against the oracle"""
    capi = gpu_lib
    rng = np.random.default_rng(11)
    bw, bg = 50, 0.003
    lengths = [int(x) for x in rng.integers(1_000, 9_000_000, size=5)]
    data = []
    with capi.Lib(0) as g:
        g.set_params(bw, 1, bg)
        for L in lengths:
            u = g.add_unit(L)
            pos, cnt = random_unit(rng, L, bw)
            g.scatter(u, 0, 0, pos, cnt[:, 0])
            data.append((pos, cnt))
        for _ in range(3):
            n = g.run()
        regs, gcnt = g.regions(n)
    for u, (pos, cnt) in enumerate(data):
        ref, ref_sums = oracle.run_unit(bw, bg, pos, cnt)
        m = regs["unit"] == u
        for k in ("left", "right", "peak", "sum", "accepted"):
            assert np.array_equal(ref[k], regs[m][k]), (u, k)
        assert np.array_equal(ref_sums, gcnt[m])
        assert ref["peak_score"].tobytes() == regs[m]["peak_score"].tobytes()



def _open(capi, launcher):
    """a context with the launcher thread on (default) or off
    (UNIPEAK_LAUNCHER=0: the caller's thread launches, K1x..K3 of a pass go
    out as a cached hipGraph keyed by every launch argument); up_open reads
    the variable"""
    import os
    old = os.environ.get("UNIPEAK_LAUNCHER")
    os.environ["UNIPEAK_LAUNCHER"] = "1" if launcher else "0"
    try:
        return capi.Lib(0)
    finally:
        if old is None:
            del os.environ["UNIPEAK_LAUNCHER"]
        else:
            os.environ["UNIPEAK_LAUNCHER"] = old


@pytest.mark.parametrize("launcher,ntargets", [(True, 2), (False, 2), (False, 9)])
def test_many_passes_rotating_targets(gpu_lib, launcher, ntargets):
    """bench-shaped: UP_MAX_IN_FLIGHT passes in flight (timing level 1) while
    this thread waits for, times and reads the older passes.  With the
    launcher thread K1x..K3 are plain launches on it; without it they are
    cached graphs -- ntargets record targets per pass slot makes 9 distinct
    graph keys per slot, past the 8-entry cache (eviction and re-capture)"""
    capi = gpu_lib
    rng = np.random.default_rng(11)
    bw = 50
    with _open(capi, launcher) as g:
        g.set_params(bw, 1, 0.003)
        _load(g, rng, [int(x) for x in rng.integers(300_000, 3_000_000, size=9)], bw)
        n = g.run()
        ref, _ = g.regions(n)
        cap = n + 16
        depth = capi.MAX_IN_FLIGHT
        bufs = [_target(cap, 1, capi.REGION_DTYPE.itemsize) for _ in range(ntargets * depth)]
        for b, off in bufs:
            g.host_register(b[off:].ctypes.data, len(b) - off)
        g.set_timing(1)
        npass = 60
        for i in range(npass + depth - 1):
            if i < npass:
                b, off = bufs[i % len(bufs)]
                g.set_record_target(b[off:].ctypes.data, cap)
                g.run_async()
            if i >= depth - 1:
                j = i - depth + 1
                assert g.run_wait() == n
                assert g.timings()[0] > 0
                b, off = bufs[j % len(bufs)]
                recs, _ = _parse(b, off, cap, 1, capi.REGION_DTYPE)
                assert recs.tobytes() == ref.tobytes()
        g.set_record_target(0, 0)
        g.set_timing(2)


@pytest.mark.parametrize("launcher", [True, False])
def test_mixed_host_delivery_and_targets(gpu_lib, launcher):
    """passes queued with host delivery (no target) and with a registered
    target alternate while UP_MAX_IN_FLIGHT passes are in flight: each pass
    keeps the delivery it was queued with (the launcher reads only the
    request snapshot), and the host view of a host-delivered pass is valid
    although a target is set for the later passes"""
    capi = gpu_lib
    rng = np.random.default_rng(23)
    bw = 50
    with _open(capi, launcher) as g:
        g.set_params(bw, 1, 0.003)
        _load(g, rng, [int(x) for x in rng.integers(200_000, 2_000_000, size=6)], bw)
        n = g.run()
        ref, rcnt = g.regions(n)
        cap = n + 16
        depth = capi.MAX_IN_FLIGHT
        bufs = [_target(cap, 1, capi.REGION_DTYPE.itemsize) for _ in range(2 * depth)]
        for b, off in bufs:
            g.host_register(b[off:].ctypes.data, len(b) - off)
        npass = 31
        host = [i % 3 == 0 for i in range(npass)]
        for i in range(npass + depth - 1):
            if i < npass:
                if host[i]:
                    g.set_record_target(0, 0)
                else:
                    b, off = bufs[i % len(bufs)]
                    g.set_record_target(b[off:].ctypes.data, cap)
                g.run_async()
            if i >= depth - 1:
                j = i - depth + 1
                assert g.run_wait() == n
                if host[j]:
                    recs, cnt = g.regions(n)
                else:
                    b, off = bufs[j % len(bufs)]
                    recs, cnt = _parse(b, off, cap, 1, capi.REGION_DTYPE)
                    with pytest.raises(capi.UpError):
                        g.regions(n)  # this pass delivered into its target
                assert recs.tobytes() == ref.tobytes(), j
                assert np.array_equal(cnt, rcnt), j
        g.set_record_target(0, 0)
