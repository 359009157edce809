"""ctypes binding of include/unipeak_hip.h (libunipeak_hip.so).

Mirrors the C-ABI one-to-one; every failing call raises UpError carrying
the library's error text (up_strerror), the analogue of the reference's
`error: ...` exits.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# UNIPEAK_LIB overrides the in-tree build (A/B experiments with variant builds)
LIB_PATH = os.environ.get("UNIPEAK_LIB") or os.path.join(_HERE, "lib", "libunipeak_hip.so")

UP_OK = 0
MAX_IN_FLIGHT = 5  # UP_MAX_IN_FLIGHT (include/unipeak_hip.h)


class UpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (code {code})")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [
        ("bw", ctypes.c_uint16),
        ("n_samples", ctypes.c_uint16),
        ("nondir", ctypes.c_int32),
        ("background", ctypes.c_double),
        ("region_thr", ctypes.c_double),
        ("kurt_thr", ctypes.c_double),
        ("corr_thr", ctypes.c_double),
        ("hit_thr", ctypes.c_double),
        ("is_control", ctypes.POINTER(ctypes.c_uint8)),
        ("coeffs", ctypes.POINTER(ctypes.c_double)),
        ("n_coeffs", ctypes.c_uint32),
        ("want_corr", ctypes.c_int32),
    ]


class Region(ctypes.Structure):
    _fields_ = [
        ("unit", ctypes.c_uint32),
        ("left", ctypes.c_uint32),
        ("right", ctypes.c_uint32),
        ("peak", ctypes.c_uint32),
        ("sum", ctypes.c_uint32),
        ("nonctl_sum", ctypes.c_uint32),
        ("accepted", ctypes.c_int32),
        ("close_pos", ctypes.c_uint32),
        ("peak_score", ctypes.c_double),
        ("kurtosis", ctypes.c_double),
        ("corr", ctypes.c_double),
    ]


REGION_DTYPE = np.dtype([
    ("unit", "<u4"), ("left", "<u4"), ("right", "<u4"), ("peak", "<u4"),
    ("sum", "<u4"), ("nonctl_sum", "<u4"), ("accepted", "<i4"), ("close_pos", "<u4"),
    ("peak_score", "<f8"), ("kurtosis", "<f8"), ("corr", "<f8")])
assert REGION_DTYPE.itemsize == ctypes.sizeof(Region)

_lib = None

EXPORTS = [
    "up_version", "up_track_bits", "up_strerror", "up_device_count", "up_kernel_weights", "up_open",
    "up_close", "up_set_params", "up_add_unit", "up_unit_count", "up_unit_pack",
    "up_unit_scatter", "up_unit_synth", "up_unit_synth_offset", "up_unit_synth_ex", "up_unit_tag_total", "up_unit_set_last_add", "up_unit_last_add",
    "up_reset_units", "up_run", "up_get_regions", "up_regions_view", "up_shift_scan", "up_shift_best",
    "up_timings", "up_scan_density", "up_unit_profile", "up_hbm_copy_gbps", "up_set_record_target",
    "up_host_register", "up_unit_profile_range", "up_run_async", "up_run_wait", "up_set_timing",
    "up_set_profile_capture", "up_unit_replay_profile",
    "up_set_index_policy", "up_invalidate_index", "up_index_state",
    "up_tir_open", "up_tir_close", "up_tir_set_stream", "up_tir_query", "up_tir_timings",
    "up_cm_open", "up_cm_close", "up_cm_add", "up_cm_collect", "up_cm_timings",
]
TIR_HOST = 0xFFFFFFFF  # UP_TIR_HOST
INDEX_AUTO, INDEX_NEVER, INDEX_ALWAYS = 0, 1, 2  # UP_INDEX_*


def load_library(path=LIB_PATH):
    """Load libunipeak_hip.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `python __graft_entry__.py` / tools/build.py")
    L = ctypes.CDLL(path)
    c = ctypes
    vp, u32p = c.c_void_p, c.POINTER(c.c_uint32)
    sig = {
        "up_version": (c.c_int, []),
        "up_track_bits": (c.c_int, []),
        "up_strerror": (c.c_char_p, [c.c_int]),
        "up_device_count": (c.c_int, [c.POINTER(c.c_int)]),
        "up_kernel_weights": (c.c_int, [c.c_uint16, c.c_double, vp]),
        "up_open": (c.c_int, [c.c_int, c.POINTER(vp)]),
        "up_close": (None, [vp]),
        "up_set_params": (c.c_int, [vp, c.POINTER(Params)]),
        "up_add_unit": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_int32, u32p]),
        "up_unit_count": (c.c_int, [vp, u32p]),
        "up_unit_pack": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16, vp]),
        "up_unit_scatter": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16, c.c_size_t, vp, vp]),
        "up_unit_synth": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16, c.c_uint64,
                                    c.c_uint32, c.c_int32, c.c_int32, c.c_int32]),
        "up_unit_synth_offset": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16, c.c_uint64,
                                           c.c_uint32, c.c_int32, c.c_int32, c.c_int32, c.c_int32]),
        "up_unit_synth_ex": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16, c.c_uint64,
                                       c.c_uint32, c.c_int32, c.c_int32, c.c_int32, c.c_int32,
                                       c.c_uint64]),
        "up_unit_tag_total": (c.c_int, [vp, c.c_uint32, c.c_int32, c.c_uint16,
                                        c.POINTER(c.c_uint64)]),
        "up_unit_set_last_add": (c.c_int, [vp, c.c_uint32, c.c_uint32]),
        "up_unit_last_add": (c.c_int, [vp, c.c_uint32, u32p]),
        "up_reset_units": (c.c_int, [vp]),
        "up_run": (c.c_int, [vp, c.POINTER(c.c_uint64)]),
        "up_run_async": (c.c_int, [vp]),
        "up_run_wait": (c.c_int, [vp, c.POINTER(c.c_uint64)]),
        "up_set_timing": (c.c_int, [vp, c.c_int]),
        "up_get_regions": (c.c_int, [vp, vp, vp, c.c_size_t]),
        "up_regions_view": (c.c_int, [vp, c.POINTER(vp), c.POINTER(vp), c.POINTER(c.c_uint64)]),
        "up_shift_scan": (c.c_int, [vp, vp, c.c_size_t, c.c_uint16, vp]),
        "up_shift_best": (c.c_int, [vp, vp, c.c_size_t, c.c_uint16, vp, vp]),
        "up_timings": (c.c_int, [vp, vp, c.c_int]),
        "up_scan_density": (c.c_int, [vp, u32p]),
        "up_set_index_policy": (c.c_int, [vp, c.c_int]),
        "up_invalidate_index": (c.c_int, [vp]),
        "up_index_state": (c.c_int, [vp, c.POINTER(c.c_int), c.POINTER(c.c_uint64)]),
        "up_unit_profile": (c.c_int, [vp, c.c_uint32, vp, vp, c.c_uint32]),
        "up_hbm_copy_gbps": (c.c_int, [vp, c.c_uint64, c.c_int, c.POINTER(c.c_double)]),
        "up_set_record_target": (c.c_int, [vp, vp, c.c_uint64]),
        "up_host_register": (c.c_int, [vp, vp, c.c_uint64]),
        "up_unit_profile_range": (c.c_int, [vp, c.c_uint32, c.c_uint64, c.c_uint32, vp, vp]),
        "up_set_profile_capture": (c.c_int, [vp, c.c_int]),
        "up_unit_replay_profile": (c.c_int, [vp, c.c_uint32, u32p, c.POINTER(c.c_uint64), vp, vp, vp,
                                             c.c_uint64]),
        "up_tir_open": (c.c_int, [c.c_int, c.POINTER(vp)]),
        "up_tir_close": (None, [vp]),
        "up_tir_set_stream": (c.c_int, [vp, c.c_uint32, c.c_uint64, vp, vp, vp]),
        "up_tir_query": (c.c_int, [vp, c.c_uint32, c.c_uint64, vp, vp, vp, vp, vp, vp, vp]),
        "up_tir_timings": (c.c_int, [vp, vp, c.c_int]),
        "up_cm_open": (c.c_int, [c.c_int, c.c_uint32, vp, c.POINTER(vp)]),
        "up_cm_close": (None, [vp]),
        "up_cm_add": (c.c_int, [vp, c.c_uint64, vp, vp, vp, vp]),
        "up_cm_collect": (c.c_int, [vp, c.c_int, c.POINTER(c.c_uint64), vp, vp, vp, vp, c.c_uint64]),
        "up_cm_timings": (c.c_int, [vp, vp, c.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _ck(code):
    if code != UP_OK:
        raise UpError(code, _lib.up_strerror(code).decode())


def kernel_weights(bw, total=1.0):
    L = load_library()
    w = np.zeros(2 * bw + 1, np.float64)
    _ck(L.up_kernel_weights(bw, total, w.ctypes.data))
    return w


def track_bits():
    """bits per stored count in a device track (up_track_bits)"""
    return load_library().up_track_bits()


def device_count():
    L = load_library()
    n = ctypes.c_int(0)
    _ck(L.up_device_count(ctypes.byref(n)))
    return n.value


# Mixing with torch: torch's bundled HIP runtime must initialise the GPU
# before this library's (system ROCm) runtime does, or torch then reports no
# GPU -- touch torch.cuda first (tools/mix_probe.py shows both orders).
class Lib:
    """One up_ctx (one GPU)."""

    def __init__(self, device=0):
        self.L = load_library()
        self.ctx = ctypes.c_void_p()
        _ck(self.L.up_open(device, ctypes.byref(self.ctx)))
        self.S = None

    def close(self):
        if self.ctx:
            self.L.up_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_params(self, bw, n_samples, background, region_thr=25.0, kurt_thr=50.0,
                   corr_thr=-1.0, hit_thr=10.0, nondir=False, control=None, coeffs=None,
                   want_corr=False):
        p = Params()
        p.bw, p.n_samples, p.nondir = bw, n_samples, int(bool(nondir))
        p.background, p.region_thr, p.kurt_thr = background, region_thr, kurt_thr
        p.corr_thr, p.hit_thr, p.want_corr = corr_thr, hit_thr, int(bool(want_corr))
        self._ctl = None
        if control is not None:
            self._ctl = (ctypes.c_uint8 * n_samples)(*[1 if x else 0 for x in control])
            p.is_control = self._ctl
        self._coef = None
        if coeffs is not None and len(coeffs):
            self._coef = (ctypes.c_double * len(coeffs))(*coeffs)
            p.coeffs = self._coef
            p.n_coeffs = len(coeffs)
        _ck(self.L.up_set_params(self.ctx, ctypes.byref(p)))
        self.S = n_samples
        self.nondir = bool(nondir)

    def add_unit(self, length, buffer_id=0):
        u = ctypes.c_uint32()
        _ck(self.L.up_add_unit(self.ctx, length, 2 if self.nondir else 1, buffer_id,
                               ctypes.byref(u)))
        return u.value

    def scatter(self, unit, strand, sample, pos, counts):
        pos = np.ascontiguousarray(pos, np.uint32)
        counts = np.ascontiguousarray(counts, np.uint32)
        assert pos.shape == counts.shape
        _ck(self.L.up_unit_scatter(self.ctx, unit, strand, sample, pos.size,
                                   pos.ctypes.data, counts.ctypes.data))

    def synth(self, unit, strand, sample, seed, contig_index, synth_strand, nondir=False,
              peaks=True, offset=0, peak_seed=0):
        """peak_seed != 0: replicate mode (shared peak centres)"""
        if peak_seed:
            _ck(self.L.up_unit_synth_ex(self.ctx, unit, strand, sample, seed, contig_index,
                                        synth_strand, int(nondir), int(peaks), int(offset),
                                        int(peak_seed)))
        elif offset:
            _ck(self.L.up_unit_synth_offset(self.ctx, unit, strand, sample, seed, contig_index,
                                            synth_strand, int(nondir), int(peaks), int(offset)))
        else:
            _ck(self.L.up_unit_synth(self.ctx, unit, strand, sample, seed, contig_index,
                                     synth_strand, int(nondir), int(peaks)))

    def tag_total(self, unit, strand, sample):
        v = ctypes.c_uint64()
        _ck(self.L.up_unit_tag_total(self.ctx, unit, strand, sample, ctypes.byref(v)))
        return v.value

    def pack(self, unit, strand, sample, dev_ptr):
        """replace a track from a device uint32 array (e.g. a torch tensor's
        data_ptr()) of contig_len counts"""
        _ck(self.L.up_unit_pack(self.ctx, unit, strand, sample, ctypes.c_void_p(dev_ptr)))

    def set_last_add(self, unit, pos):
        _ck(self.L.up_unit_set_last_add(self.ctx, unit, pos))

    def last_add(self, unit):
        v = ctypes.c_uint32()
        _ck(self.L.up_unit_last_add(self.ctx, unit, ctypes.byref(v)))
        return v.value

    def reset_units(self):
        _ck(self.L.up_reset_units(self.ctx))

    def run(self):
        n = ctypes.c_uint64()
        _ck(self.L.up_run(self.ctx, ctypes.byref(n)))
        return n.value

    def run_async(self):
        """enqueue one pass (at most MAX_IN_FLIGHT in flight); see up_run_async"""
        _ck(self.L.up_run_async(self.ctx))

    def run_wait(self):
        """complete the oldest pass in flight -> its region count"""
        n = ctypes.c_uint64()
        _ck(self.L.up_run_wait(self.ctx, ctypes.byref(n)))
        return n.value

    def set_timing(self, level):
        """0: wall only, 1: + K1a events, 2: every phase (default)"""
        _ck(self.L.up_set_timing(self.ctx, int(level)))

    def regions(self, n, with_counts=True):
        out = np.zeros(n, REGION_DTYPE)
        cnt = np.zeros((n, self.S), np.uint32) if with_counts else None
        _ck(self.L.up_get_regions(self.ctx, out.ctypes.data,
                                  cnt.ctypes.data if cnt is not None else None, n))
        return out, cnt

    def regions_view(self):
        """(records, counts) as numpy views of the context's pinned host copy;
        valid until the next run()."""
        r, k, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        _ck(self.L.up_regions_view(self.ctx, ctypes.byref(r), ctypes.byref(k), ctypes.byref(n)))
        n = n.value
        if n == 0:
            return np.zeros(0, REGION_DTYPE), np.zeros((0, self.S), np.uint32)
        regs = np.frombuffer((ctypes.c_char * (n * REGION_DTYPE.itemsize)).from_address(r.value),
                             REGION_DTYPE)
        cnt = np.frombuffer((ctypes.c_char * (n * self.S * 4)).from_address(k.value),
                            np.uint32).reshape(n, self.S)
        return regs, cnt

    def shift_scan(self, idx, max_shift):
        idx = np.ascontiguousarray(idx, np.uint64)
        out = np.zeros((idx.size, max_shift + 1), np.float64)
        _ck(self.L.up_shift_scan(self.ctx, idx.ctypes.data, idx.size, max_shift,
                                 out.ctypes.data))
        return out

    def shift_best(self, idx, max_shift):
        """-> (best shift uint16[n], best corr f8[n]) per region (up_shift_best)"""
        idx = np.ascontiguousarray(idx, np.uint64)
        best = np.zeros(idx.size, np.uint16)
        corr = np.zeros(idx.size, np.float64)
        _ck(self.L.up_shift_best(self.ctx, idx.ctypes.data, idx.size, max_shift, best.ctypes.data,
                                 corr.ctypes.data))
        return best, corr

    def set_record_target(self, dev_ptr, cap):
        """records of the next runs go to a device buffer (see the header);
        dev_ptr = 0 restores host delivery"""
        _ck(self.L.up_set_record_target(self.ctx, ctypes.c_void_p(dev_ptr or None), cap))

    def host_register(self, ptr, nbytes):
        _ck(self.L.up_host_register(self.ctx, ctypes.c_void_p(ptr), nbytes))

    def hbm_copy_gbps(self, nbytes=1 << 30, reps=5):
        v = ctypes.c_double()
        _ck(self.L.up_hbm_copy_gbps(self.ctx, nbytes, reps, ctypes.byref(v)))
        return v.value

    def set_index_policy(self, policy):
        """INDEX_AUTO / INDEX_NEVER / INDEX_ALWAYS (up_set_index_policy)"""
        _ck(self.L.up_set_index_policy(self.ctx, int(policy)))

    def invalidate_index(self):
        _ck(self.L.up_invalidate_index(self.ctx))

    def index_state(self):
        """(the next pass uses the index, index builds so far)"""
        on, b = ctypes.c_int(0), ctypes.c_uint64(0)
        _ck(self.L.up_index_state(self.ctx, ctypes.byref(on), ctypes.byref(b)))
        return bool(on.value), int(b.value)

    def scan_density(self):
        """bytes K1a streams per 1,024 positions of a unit (up_scan_density)"""
        v = ctypes.c_uint32()
        _ck(self.L.up_scan_density(self.ctx, ctypes.byref(v)))
        return v.value

    def timings(self):
        t = np.zeros(5, np.float64)
        _ck(self.L.up_timings(self.ctx, t.ctypes.data, 5))
        return t

    def profile(self, unit, length):
        f = np.zeros(length, np.float64)
        r = np.zeros(length, np.float64)
        _ck(self.L.up_unit_profile(self.ctx, unit, f.ctypes.data, r.ctypes.data, length))
        return f, r

    def set_profile_capture(self, on):
        _ck(self.L.up_set_profile_capture(self.ctx, int(bool(on))))

    def replay_profile(self, unit):
        """(resync, event[], pos[], score[]) of a replayed unit (up_unit_replay_profile)"""
        rs, n = ctypes.c_uint32(), ctypes.c_uint64()
        _ck(self.L.up_unit_replay_profile(self.ctx, unit, ctypes.byref(rs), ctypes.byref(n), None, None,
                                          None, 0))
        ev = np.zeros(n.value, np.uint32)
        pos = np.zeros(n.value, np.uint32)
        sc = np.zeros(n.value, np.float64)
        if n.value:
            _ck(self.L.up_unit_replay_profile(self.ctx, unit, ctypes.byref(rs), ctypes.byref(n),
                                              ev.ctypes.data, pos.ctypes.data, sc.ctypes.data, n.value))
        return rs.value, ev, pos, sc


class Tir:
    """One up_tir handle: tags_in_regions' streams and queries on one GPU."""

    def __init__(self, device=0):
        self.L = load_library()
        self.h = ctypes.c_void_p()
        _ck(self.L.up_tir_open(device, ctypes.byref(self.h)))
        self.n = 0

    def close(self):
        if self.h:
            self.L.up_tir_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, idx, contig, first, count, forward):
        key = (np.asarray(contig, np.uint64) << np.uint64(32)) | np.asarray(first, np.uint64)
        cnt = np.ascontiguousarray(count, np.uint32)
        fwd = np.ascontiguousarray(forward, np.uint8)
        _ck(self.L.up_tir_set_stream(self.h, idx, len(key), key.ctypes.data, cnt.ctypes.data,
                                     fwd.ctypes.data))
        self.n = max(self.n, idx + 1)

    def query(self, contig, left, right, forward, n_streams=None):
        """(first, end, hits), each [R][n_streams] uint32"""
        S = n_streams or self.n
        rc = np.ascontiguousarray(contig, np.uint32)
        rl = np.ascontiguousarray(left, np.uint32)
        rr = np.ascontiguousarray(right, np.uint32)
        rf = np.ascontiguousarray(forward, np.uint8)
        R = len(rc)
        out = [np.zeros((R, S), np.uint32) for _ in range(3)]
        _ck(self.L.up_tir_query(self.h, S, R, rc.ctypes.data, rl.ctypes.data, rr.ctypes.data,
                                rf.ctypes.data, *(o.ctypes.data for o in out)))
        return tuple(out)

    def timings(self):
        t = np.zeros(2, np.float64)
        _ck(self.L.up_tir_timings(self.h, t.ctypes.data, 2))
        return t


class CountMap:
    """One up_cm handle: convert_align's CountMap as dense HBM tracks."""

    def __init__(self, contig_lens, device=0):
        self.L = load_library()
        self.h = ctypes.c_void_p()
        lens = np.ascontiguousarray(contig_lens, np.uint32)
        _ck(self.L.up_cm_open(device, len(lens), lens.ctypes.data, ctypes.byref(self.h)))

    def close(self):
        if self.h:
            self.L.up_cm_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def add(self, contig, pos, forward, count=None):
        c = np.ascontiguousarray(contig, np.uint32)
        p = np.ascontiguousarray(pos, np.uint32)
        f = np.ascontiguousarray(forward, np.uint8)
        k = None if count is None else np.ascontiguousarray(count, np.uint32)
        _ck(self.L.up_cm_add(self.h, len(p), c.ctypes.data, p.ctypes.data, f.ctypes.data,
                             None if k is None else k.ctypes.data))

    def collect(self, nondir=False):
        """(contig, pos, count, forward) in the iterators' order"""
        n = ctypes.c_uint64()
        _ck(self.L.up_cm_collect(self.h, int(nondir), ctypes.byref(n), None, None, None, None, 0))
        out = [np.zeros(n.value, np.uint32) for _ in range(3)] + [np.zeros(n.value, np.uint8)]
        if n.value:
            _ck(self.L.up_cm_collect(self.h, int(nondir), ctypes.byref(n), *(o.ctypes.data for o in out),
                                     n.value))
        return tuple(out)
