"""ctypes binding of the oracle (TEST INFRASTRUCTURE: CPU restatement of the
reference path, oracle/orc.h).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline use it."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class UnitRegion(ctypes.Structure):
    _fields_ = [("left", ctypes.c_uint32), ("right", ctypes.c_uint32),
                ("peak", ctypes.c_uint32), ("npos", ctypes.c_uint32),
                ("contig", ctypes.c_uint32), ("forward", ctypes.c_int32),
                ("accepted", ctypes.c_int32), ("sum", ctypes.c_uint32),
                ("peak_score", ctypes.c_double), ("kurtosis", ctypes.c_double),
                ("corr", ctypes.c_double)]


UNIT_DTYPE = np.dtype([("left", "<u4"), ("right", "<u4"), ("peak", "<u4"), ("npos", "<u4"),
                       ("contig", "<u4"), ("forward", "<i4"), ("accepted", "<i4"),
                       ("sum", "<u4"), ("peak_score", "<f8"), ("kurtosis", "<f8"),
                       ("corr", "<f8")])
assert UNIT_DTYPE.itemsize == ctypes.sizeof(UnitRegion)


class Oracle:
    def __init__(self, path=ORACLE_LIB):
        L = ctypes.CDLL(path)
        vp, c = ctypes.c_void_p, ctypes
        L.orc_kernel.argtypes = [c.c_uint16, c.c_double, vp]
        L.orc_kernel.restype = None
        L.orc_run_unit.restype = c.c_int64
        L.orc_run_unit.argtypes = [vp, c.c_uint32, c.c_double, c.c_double, c.c_double,
                                   c.c_double, c.c_int, c.c_int, c.c_uint16, vp, vp,
                                   c.c_uint32, c.c_uint32, c.c_size_t, vp, vp, vp, vp, vp,
                                   c.c_size_t]
        L.orc_unit_profile.restype = c.c_int
        L.orc_unit_profile.argtypes = [vp, c.c_uint32, c.c_int, c.c_int, c.c_uint16, vp, vp,
                                       c.c_uint32, c.c_size_t, vp, vp, vp, c.c_uint32, vp]
        L.orc_synth_track.restype = c.c_size_t
        L.orc_synth_track.argtypes = [c.c_uint64, c.c_uint32, c.c_int, c.c_int, c.c_uint32,
                                      c.c_uint16, c.c_int, vp, vp, c.c_size_t]
        L.orc_synth_track_ex.restype = c.c_size_t
        L.orc_synth_track_ex.argtypes = [c.c_uint64, c.c_uint32, c.c_int, c.c_int, c.c_uint32,
                                         c.c_uint16, c.c_int, c.c_int32, c.c_uint64, vp, vp,
                                         c.c_size_t]
        L.orc_genome_unit.restype = c.c_int64
        L.orc_genome_unit.argtypes = [vp, c.c_uint32, c.c_double, c.c_double, c.c_double,
                                      c.c_double, c.c_int, c.c_int, c.c_uint16, vp, vp, vp,
                                      c.c_uint64, vp, c.c_uint32, c.c_uint32, c.c_uint16, vp, vp,
                                      c.c_size_t]
        L.orc_baseline_run.restype = c.c_int
        L.orc_baseline_run.argtypes = [c.c_uint32, vp, c.c_uint64, c.c_uint16, c.c_double,
                                       c.c_double, c.c_double, c.c_double, vp, vp, vp]
        L.orc_baseline_unit.restype = c.c_int
        L.orc_baseline_unit.argtypes = [vp, vp, c.c_size_t, c.c_uint32, c.c_int, c.c_uint16,
                                        c.c_double, c.c_double, c.c_double, c.c_double, vp, vp]
        L.orc_format_pairs.restype = c.c_size_t
        L.orc_format_pairs.argtypes = [vp, vp, c.c_size_t, c.c_int, vp]
        self.L = L

    def kernel(self, bw, total):
        w = np.zeros(2 * bw + 1, np.float64)
        self.L.orc_kernel(bw, total, w.ctypes.data)
        return w

    @staticmethod
    def _opt(a, dt):
        return None if a is None else np.ascontiguousarray(a, dt)

    def run_unit(self, bw, background, pos, counts_fwd, counts_rev=None, *, region_thr=25.0,
                 kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0, buffer_forward=True,
                 nondir=False, control=None, coeffs=None, contig=0, cap=1 << 16):
        """All candidate regions (accepted and rejected) of one unit."""
        k = self.kernel(bw, 1.0 / background)
        pos = np.ascontiguousarray(pos, np.uint32)
        S = counts_fwd.shape[1] if counts_fwd is not None else counts_rev.shape[1]
        cf = self._opt(counts_fwd, np.uint32)
        cr = self._opt(counts_rev, np.uint32)
        ctl = np.zeros(S, np.uint8) if control is None else np.asarray(control, np.uint8)
        co = self._opt(coeffs, np.float64)
        out = np.zeros(cap, UNIT_DTYPE)
        sums = np.zeros((cap, S), np.uint32)
        n = self.L.orc_run_unit(k.ctypes.data, k.size, region_thr, kurt_thr, corr_thr, hit_thr,
                                int(buffer_forward), int(nondir), S, ctl.ctypes.data,
                                None if co is None else co.ctypes.data,
                                0 if co is None else co.size, contig, pos.size, pos.ctypes.data,
                                None if cf is None else cf.ctypes.data,
                                None if cr is None else cr.ctypes.data,
                                out.ctypes.data, sums.ctypes.data, cap)
        assert n <= cap
        return out[:n], sums[:n]

    def profile(self, bw, background, length, pos, counts_fwd, counts_rev=None, *,
                buffer_forward=True, nondir=False, control=None, coeffs=None):
        k = self.kernel(bw, 1.0 / background)
        pos = np.ascontiguousarray(pos, np.uint32)
        S = counts_fwd.shape[1] if counts_fwd is not None else counts_rev.shape[1]
        cf = self._opt(counts_fwd, np.uint32)
        cr = self._opt(counts_rev, np.uint32)
        ctl = np.zeros(S, np.uint8) if control is None else np.asarray(control, np.uint8)
        co = self._opt(coeffs, np.float64)
        out = np.zeros(length, np.float64)
        self.L.orc_unit_profile(k.ctypes.data, k.size, int(buffer_forward), int(nondir), S,
                                ctl.ctypes.data, None if co is None else co.ctypes.data,
                                0 if co is None else co.size, pos.size, pos.ctypes.data,
                                None if cf is None else cf.ctypes.data,
                                None if cr is None else cr.ctypes.data, length, out.ctypes.data)
        return out

    def synth_track(self, seed, contig, strand, nondir, length, bw, peaks=True):
        cap = length // 40 + 4096
        pos = np.zeros(cap, np.uint32)
        cnt = np.zeros(cap, np.uint32)
        n = self.L.orc_synth_track(seed, contig, strand, int(nondir), length, bw, int(peaks),
                                   pos.ctypes.data, cnt.ctypes.data, cap)
        assert n <= cap
        return pos[:n].copy(), cnt[:n].copy()

    def synth_track_ex(self, seed, contig, strand, nondir, length, bw, peaks=True, offset=0,
                       peak_seed=0):
        n = self.L.orc_synth_track_ex(seed, contig, strand, int(nondir), length, bw, int(peaks),
                                      offset, peak_seed, None, None, 0)
        pos = np.zeros(n + 1, np.uint32)
        cnt = np.zeros(n + 1, np.uint32)
        m = self.L.orc_synth_track_ex(seed, contig, strand, int(nondir), length, bw, int(peaks),
                                      offset, peak_seed, pos.ctypes.data, cnt.ctypes.data, n + 1)
        assert m == n
        return pos[:n].copy(), cnt[:n].copy()

    def genome_unit(self, bw, background, contig, length, seeds, with_peaks, *, region_thr=25.0,
                    kurt_thr=50.0, corr_thr=-1.0, hit_thr=10.0, buffer_forward=True,
                    nondir=False, control=None, peak_seed=0, offset=(0, 0), cap=1 << 20):
        """All candidate regions of one synthetic unit, generated and run
        inside the oracle (orc_genome_unit): no host count matrices."""
        k = self.kernel(bw, 1.0 / background)
        S = len(seeds)
        sd = np.ascontiguousarray(seeds, np.uint64)
        wp = np.ascontiguousarray(with_peaks, np.uint8)
        ctl = np.zeros(S, np.uint8) if control is None else np.asarray(control, np.uint8)
        off = np.ascontiguousarray(offset, np.int32)
        out = np.zeros(cap, UNIT_DTYPE)
        sums = np.zeros((cap, S), np.uint32)
        n = self.L.orc_genome_unit(k.ctypes.data, k.size, region_thr, kurt_thr, corr_thr, hit_thr,
                                   int(buffer_forward), int(nondir), S, ctl.ctypes.data,
                                   sd.ctypes.data, wp.ctypes.data, peak_seed, off.ctypes.data,
                                   contig, length, bw, out.ctypes.data, sums.ctypes.data, cap)
        assert n <= cap
        return out[:n], sums[:n]

    def baseline(self, lens, seed, bw, region_thr, kurt_thr, hit_thr, background):
        lens = np.ascontiguousarray(lens, np.uint32)
        npass = ctypes.c_uint64()
        nrej = ctypes.c_uint64()
        sec = ctypes.c_double()
        self.L.orc_baseline_run(lens.size, lens.ctypes.data, seed, bw, region_thr, kurt_thr,
                                hit_thr, background, ctypes.byref(npass), ctypes.byref(nrej),
                                ctypes.byref(sec))
        return npass.value, nrej.value, sec.value

    def baseline_unit(self, pos, cnt, contig, strand, bw, region_thr, kurt_thr, hit_thr,
                      background):
        """one (contig, strand) unit of the hot-path baseline over given hits
        -> (pass, reject)"""
        pos = np.ascontiguousarray(pos, np.uint32)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        npass = ctypes.c_uint64()
        nrej = ctypes.c_uint64()
        self.L.orc_baseline_unit(pos.ctypes.data, cnt.ctypes.data, pos.size, contig, strand, bw,
                                 region_thr, kurt_thr, hit_thr, background, ctypes.byref(npass),
                                 ctypes.byref(nrej))
        return npass.value, nrej.value

    def format_pairs(self, pos, cnt, neg):
        """wiggle data lines for (pos, count) pairs as bytes"""
        pos = np.ascontiguousarray(pos, np.uint32)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        buf = np.empty(pos.size * 24 + 1, np.uint8)
        n = self.L.orc_format_pairs(pos.ctypes.data, cnt.ctypes.data, pos.size, int(bool(neg)),
                                    buf.ctypes.data)
        return buf[:n].tobytes()
