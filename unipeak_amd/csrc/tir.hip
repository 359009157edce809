// unipeak_amd/csrc/tir.hip -- bin/tags_in_regions on the GPU (SURVEY.md
// 8(f)3; include/unipeak_hip.h "tags_in_regions").
//
// The reference (src/tags_in_regions.cpp:181-195) walks one cursor per
// sample through that sample's alignment stream, region by region: skip
// records until one has the region's strand and (contig, firstPos) >=
// (contig, left), then add up counts while the record is on the contig at
// firstPos <= right -- whatever its strand (quirk Q12).  Each region's answer
// depends on where the previous region left the cursor, so the device
// answers every (region, stream) pair as if the cursor started at the
// stream's first record ("speculative"), in parallel, and the host keeps the
// answer wherever the real cursor has not passed the speculative start --
// then nothing in between qualifies, and the two walks are identical (the
// proof is in DESIGN.md).  The host walks the rest itself.
//
// Per stream the device keeps, built by three scan launches:
//   key[i] = contig << 32 | firstPos        the record's sort key
//   psum[i] = sum of count[0..i) (uint32, wrapping like HitCount)
//   run_end[i] = end of the maximal non-decreasing run of keys holding i
//   next_f[i] / next_r[i] = first j >= i with a forward / reverse record
// so a skip is one binary search per run it crosses (plus a next_* lookup)
// and a count loop is one binary search per run plus two psum reads.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/unipeak_hip.h"

namespace {

constexpr int kThreads = 256;              // prep kernels: threads per block
constexpr int kPer = 4;                    // records per thread
constexpr int kBlock = kThreads * kPer;    // records per block
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kRunBudget = 48;             // runs one query may cross before the host takes it

struct StreamView {
    const uint64_t *key;
    const uint8_t *fwd;
    const uint32_t *psum;      // [n + 1]
    const uint32_t *run_end;   // [n]
    const uint32_t *next_f;    // [n + 1]
    const uint32_t *next_r;    // [n + 1]
    uint32_t n;
    uint32_t pad;
};

// inclusive wave scans over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}
// inclusive suffix minimum: min over lanes >= lane
__device__ __forceinline__ uint32_t wave_suffix_min(uint32_t v, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_down((int)v, d, 64);
        if (lane + d < 64) v = min(v, t);
    }
    return v;
}

// Block-local pass: every block of kBlock records writes its local exclusive
// count prefix and its local "next" indices (kNone where the answer lies in a
// later block), plus the block's aggregates for tir_blocks.
__global__ void __launch_bounds__(kThreads) tir_local(const uint64_t *__restrict__ key,
                                                      const uint32_t *__restrict__ cnt,
                                                      const uint8_t *__restrict__ fwd, uint32_t n,
                                                      uint32_t *__restrict__ psum,
                                                      uint32_t *__restrict__ run_end,
                                                      uint32_t *__restrict__ next_f,
                                                      uint32_t *__restrict__ next_r,
                                                      uint32_t *__restrict__ agg) {
    __shared__ uint32_t s_sum[kThreads / 64], s_brk[kThreads / 64], s_f[kThreads / 64],
        s_r[kThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kBlock;
    const uint64_t i0 = base + (uint64_t)tid * kPer;
    uint32_t c[kPer], brk[kPer], f[kPer], r[kPer];
    uint64_t prev = 0;
    if (i0 > 0 && i0 <= n) prev = key[i0 - 1];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint64_t i = i0 + k;
        if (i < n) {
            const uint64_t kk = key[i];
            c[k] = cnt[i];
            brk[k] = (i > 0 && kk < prev) ? (uint32_t)i : kNone;  // i starts a run
            const bool fw = fwd[i] != 0;
            f[k] = fw ? (uint32_t)i : kNone;
            r[k] = fw ? kNone : (uint32_t)i;
            prev = kk;
        } else {
            c[k] = 0;
            brk[k] = f[k] = r[k] = kNone;
        }
    }
    // thread totals
    uint32_t tsum = 0, tbrk = kNone, tf = kNone, tr = kNone;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        tsum += c[k];
        tbrk = min(tbrk, brk[k]);
        tf = min(tf, f[k]);
        tr = min(tr, r[k]);
    }
    const uint32_t isum = wave_incl_sum(tsum, lane);
    const uint32_t ibrk = wave_suffix_min(tbrk, lane);
    const uint32_t iff = wave_suffix_min(tf, lane);
    const uint32_t irr = wave_suffix_min(tr, lane);
    if (lane == 63) s_sum[wave] = isum;
    if (lane == 0) {
        s_brk[wave] = ibrk;
        s_f[wave] = iff;
        s_r[wave] = irr;
    }
    __syncthreads();
    // what the threads before / after this one contribute
    uint32_t before = isum - tsum;
    uint32_t after_brk = (uint32_t)__shfl_down((int)ibrk, 1, 64);
    uint32_t after_f = (uint32_t)__shfl_down((int)iff, 1, 64);
    uint32_t after_r = (uint32_t)__shfl_down((int)irr, 1, 64);
    if (lane == 63) after_brk = after_f = after_r = kNone;
    for (int w = 0; w < kThreads / 64; ++w) {
        if (w < wave) before += s_sum[w];
        if (w > wave) {
            after_brk = min(after_brk, s_brk[w]);
            after_f = min(after_f, s_f[w]);
            after_r = min(after_r, s_r[w]);
        }
    }
    // per record: exclusive prefix; strictly-later run start; inclusive nexts
    uint32_t run = before;
    uint32_t nb = after_brk, nf = after_f, nr = after_r;
    uint32_t o_brk[kPer], o_f[kPer], o_r[kPer];
#pragma unroll
    for (int k = kPer - 1; k >= 0; --k) {
        o_brk[k] = nb;              // starts strictly after record k
        nb = min(nb, brk[k]);
        nf = min(nf, f[k]);
        nr = min(nr, r[k]);
        o_f[k] = nf;
        o_r[k] = nr;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint64_t i = i0 + k;
        if (i < n) {
            psum[i] = run;
            run_end[i] = o_brk[k];
            next_f[i] = o_f[k];
            next_r[i] = o_r[k];
        }
        run += c[k];
    }
    if (tid == kThreads - 1) {
        agg[4 * blockIdx.x + 0] = run;  // block total
    }
    if (tid == 0) {
        uint32_t b = kNone, ff = kNone, rr = kNone;
        for (int w = 0; w < kThreads / 64; ++w) {
            b = min(b, s_brk[w]);
            ff = min(ff, s_f[w]);
            rr = min(rr, s_r[w]);
        }
        agg[4 * blockIdx.x + 1] = b;
        agg[4 * blockIdx.x + 2] = ff;
        agg[4 * blockIdx.x + 3] = rr;
    }
}

// One block: exclusive prefix of the block totals and, per block, the
// minimum of each "next" aggregate over the blocks after it (in place).
__global__ void __launch_bounds__(1024) tir_blocks(uint32_t *__restrict__ agg, uint32_t nblk,
                                                   uint32_t n, uint32_t *__restrict__ total) {
    __shared__ uint32_t s_carry[4];
    __shared__ uint32_t s_w[16][4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) {
        s_carry[0] = 0;
        s_carry[1] = s_carry[2] = s_carry[3] = n;
    }
    __syncthreads();
    // forward chunks for the sum
    for (uint32_t b0 = 0; b0 < nblk; b0 += 1024) {
        const uint32_t b = b0 + tid;
        const uint32_t v = b < nblk ? agg[4 * b] : 0;
        const uint32_t inc = wave_incl_sum(v, lane);
        if (lane == 63) s_w[wave][0] = inc;
        __syncthreads();
        uint32_t before = s_carry[0] + inc - v;
        for (int w = 0; w < wave; ++w) before += s_w[w][0];
        __syncthreads();
        if (b < nblk) agg[4 * b] = before;
        if (tid == 1023) s_carry[0] = before + v;
        __syncthreads();
    }
    if (tid == 0) *total = s_carry[0];
    // backward chunks for the minima (exclusive: blocks strictly after b)
    const uint32_t nchunk = (nblk + 1023) / 1024;
    for (int32_t ch = (int32_t)nchunk - 1; ch >= 0; --ch) {
        const uint32_t b = (uint32_t)ch * 1024 + tid;
        uint32_t v[3], inc[3];
        for (int k = 0; k < 3; ++k) {
            v[k] = b < nblk ? agg[4 * b + 1 + k] : kNone;
            inc[k] = wave_suffix_min(v[k], lane);
        }
        if (lane == 0)
            for (int k = 0; k < 3; ++k) s_w[wave][1 + k] = inc[k];
        __syncthreads();
        uint32_t out[3];
        for (int k = 0; k < 3; ++k) {
            uint32_t a = (uint32_t)__shfl_down((int)inc[k], 1, 64);
            if (lane == 63) a = kNone;
            for (int w = wave + 1; w < 16; ++w) a = min(a, s_w[w][1 + k]);
            out[k] = min(a, s_carry[1 + k]);
        }
        __syncthreads();
        if (b < nblk)
            for (int k = 0; k < 3; ++k) agg[4 * b + 1 + k] = out[k];
        if (tid == 0)
            for (int k = 0; k < 3; ++k) s_carry[1 + k] = min(out[k], v[k]);
        __syncthreads();
    }
}

// apply the block carries; the "none" answers become n (end of stream)
__global__ void __launch_bounds__(kThreads) tir_fix(uint32_t n, const uint32_t *__restrict__ agg,
                                                    const uint32_t *__restrict__ total,
                                                    uint32_t *__restrict__ psum,
                                                    uint32_t *__restrict__ run_end,
                                                    uint32_t *__restrict__ next_f,
                                                    uint32_t *__restrict__ next_r) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        psum[n] = *total;
        next_f[n] = next_r[n] = n;
        return;
    }
    const uint32_t b = (uint32_t)(i / kBlock);
    psum[i] += agg[4 * b];
    uint32_t v = run_end[i];
    run_end[i] = v != kNone ? v : min(agg[4 * b + 1], n);
    v = next_f[i];
    next_f[i] = v != kNone ? v : min(agg[4 * b + 2], n);
    v = next_r[i];
    next_r[i] = v != kNone ? v : min(agg[4 * b + 3], n);
}

// first index in [lo, hi) whose key is >= k (keys non-decreasing there)
__device__ __forceinline__ uint32_t lower_key(const uint64_t *key, uint32_t lo, uint32_t hi,
                                              uint64_t k) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (key[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// first index in [lo, hi) whose key is > k
__device__ __forceinline__ uint32_t upper_key(const uint64_t *key, uint32_t lo, uint32_t hi,
                                              uint64_t k) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (key[mid] <= k) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One thread per (region, stream): the reference's skip and count loops
// (tags_in_regions.cpp:185-190) from the stream's first record.
__global__ void __launch_bounds__(256) tir_query(const StreamView *__restrict__ sv, uint32_t S,
                                                 uint64_t R, const uint32_t *__restrict__ contig,
                                                 const uint32_t *__restrict__ left,
                                                 const uint32_t *__restrict__ right,
                                                 const uint8_t *__restrict__ fwd,
                                                 uint32_t *__restrict__ first,
                                                 uint32_t *__restrict__ end,
                                                 uint32_t *__restrict__ hits) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= R * S) return;
    const uint64_t r = t / S;
    const StreamView v = sv[t % S];
    const uint64_t c = contig[r];
    const bool fw = fwd[r] != 0;
    const uint64_t kl = c << 32 | left[r], kr = c << 32 | right[r];
    const uint32_t *nx = fw ? v.next_f : v.next_r;
    int budget = kRunBudget;
    // skip: first record with the region's strand and key >= (contig, left)
    uint32_t s = v.n;
    for (uint32_t i = 0; i < v.n;) {
        if (--budget < 0) {
            first[t] = end[t] = UP_TIR_HOST;
            hits[t] = 0;
            return;
        }
        const uint32_t e = v.run_end[i];
        const uint32_t j = lower_key(v.key, i, e, kl);
        if (j < e) {
            const uint32_t k = nx[j];
            if (k < e) {
                s = k;
                break;
            }
        }
        i = e;
    }
    // count: records on the contig at firstPos <= right, any strand (Q12)
    uint32_t e = s;
    while (e < v.n) {
        const uint64_t k = v.key[e];
        if ((k >> 32) != c || k > kr) break;
        if (--budget < 0) {
            first[t] = end[t] = UP_TIR_HOST;
            hits[t] = 0;
            return;
        }
        const uint32_t re = v.run_end[e];
        const uint32_t u = upper_key(v.key, e + 1, re, kr);
        e = u;
        if (u < re) break;
    }
    first[t] = s;
    end[t] = e;
    hits[t] = v.psum[e] - v.psum[s];
}

template <typename T>
struct Dev {
    T *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        const size_t cap = want < 16 ? 16 : want;
        hipError_t e = hipMalloc(&p, cap * sizeof(T));
        if (e == hipSuccess) n = cap;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct DevStream {
    uint32_t n = 0;
    bool ready = false;
    Dev<uint64_t> key;
    Dev<uint8_t> fwd;
    Dev<uint32_t> cnt, psum, run_end, next_f, next_r, agg, total;
    void release() {
        key.release();
        fwd.release();
        cnt.release();
        psum.release();
        run_end.release();
        next_f.release();
        next_r.release();
        agg.release();
        total.release();
        ready = false;
    }
};

}  // namespace

struct up_tir {
    int dev = 0;
    hipStream_t stream = nullptr;
    std::vector<DevStream> streams;
    Dev<StreamView> d_views;
    Dev<uint32_t> d_rc, d_rl, d_rr, d_first, d_end, d_hits;
    Dev<uint8_t> d_rf;
    float last_ms[2] = {0, 0};  // [0] stream preparation (all set_stream), [1] last query
    hipEvent_t ev[2] = {};
};

#define TIRCHK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? UP_E_NOMEM : UP_E_HIP; \
    } while (0)

extern "C" {

int up_tir_open(int hip_device, up_tir **out) {
    if (!out) return UP_E_ARG;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd < 1) return UP_E_NODEV;
    if (hip_device < 0 || hip_device >= nd) return UP_E_ARG;
    up_tir *h = new up_tir;
    h->dev = hip_device;
    if (hipSetDevice(hip_device) != hipSuccess ||
        hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev[0]) != hipSuccess || hipEventCreate(&h->ev[1]) != hipSuccess) {
        delete h;
        return UP_E_HIP;
    }
    *out = h;
    return UP_OK;
}

void up_tir_close(up_tir *h) {
    if (!h) return;
    (void)hipSetDevice(h->dev);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto &s : h->streams) s.release();
    h->d_views.release();
    h->d_rc.release();
    h->d_rl.release();
    h->d_rr.release();
    h->d_rf.release();
    h->d_first.release();
    h->d_end.release();
    h->d_hits.release();
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int up_tir_set_stream(up_tir *h, uint32_t stream, uint64_t n, const uint64_t *key,
                      const uint32_t *count, const uint8_t *forward) {
    if (!h || stream >= 4096 || n >= 0xFFFFFFFFull || (n && (!key || !count || !forward)))
        return UP_E_ARG;
    TIRCHK(hipSetDevice(h->dev));
    if (h->streams.size() <= stream) h->streams.resize(stream + 1);
    DevStream &d = h->streams[stream];
    d.n = (uint32_t)n;
    const uint32_t nblk = (uint32_t)((n + kBlock - 1) / kBlock);
    TIRCHK(d.key.ensure(n));
    TIRCHK(d.fwd.ensure(n));
    TIRCHK(d.cnt.ensure(n));
    TIRCHK(d.psum.ensure(n + 1));
    TIRCHK(d.run_end.ensure(n + 1));
    TIRCHK(d.next_f.ensure(n + 1));
    TIRCHK(d.next_r.ensure(n + 1));
    TIRCHK(d.agg.ensure(4ull * nblk + 4));
    TIRCHK(d.total.ensure(1));
    hipStream_t st = h->stream;
    if (n) {
        TIRCHK(hipMemcpyAsync(d.key.p, key, n * sizeof(uint64_t), hipMemcpyHostToDevice, st));
        TIRCHK(hipMemcpyAsync(d.cnt.p, count, n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        TIRCHK(hipMemcpyAsync(d.fwd.p, forward, n, hipMemcpyHostToDevice, st));
    }
    TIRCHK(hipEventRecord(h->ev[0], st));
    if (nblk) {
        hipLaunchKernelGGL(tir_local, dim3(nblk), dim3(kThreads), 0, st, d.key.p, d.cnt.p, d.fwd.p,
                           (uint32_t)n, d.psum.p, d.run_end.p, d.next_f.p, d.next_r.p, d.agg.p);
        TIRCHK(hipGetLastError());
        hipLaunchKernelGGL(tir_blocks, dim3(1), dim3(1024), 0, st, d.agg.p, nblk, (uint32_t)n,
                           d.total.p);
        TIRCHK(hipGetLastError());
    } else {
        TIRCHK(hipMemsetAsync(d.total.p, 0, sizeof(uint32_t), st));
    }
    const uint32_t nfix = (uint32_t)((n + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(tir_fix, dim3(nfix), dim3(kThreads), 0, st, (uint32_t)n, d.agg.p, d.total.p,
                       d.psum.p, d.run_end.p, d.next_f.p, d.next_r.p);
    TIRCHK(hipGetLastError());
    TIRCHK(hipEventRecord(h->ev[1], st));
    TIRCHK(hipStreamSynchronize(st));  // the caller's host arrays may go away
    float ms = 0;
    TIRCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->last_ms[0] = ms;
    d.ready = true;
    return UP_OK;
}

int up_tir_query(up_tir *h, uint32_t n_streams, uint64_t n_regions, const uint32_t *contig,
                 const uint32_t *left, const uint32_t *right, const uint8_t *forward,
                 uint32_t *first, uint32_t *end, uint32_t *hits) {
    if (!h || n_streams == 0 || n_streams > h->streams.size()) return UP_E_ARG;
    if (n_regions && (!contig || !left || !right || !forward || !first || !end || !hits))
        return UP_E_ARG;
    for (uint32_t s = 0; s < n_streams; ++s)
        if (!h->streams[s].ready) return UP_E_STATE;
    if (n_regions == 0) return UP_OK;
    TIRCHK(hipSetDevice(h->dev));
    std::vector<StreamView> views(n_streams);
    for (uint32_t s = 0; s < n_streams; ++s) {
        const DevStream &d = h->streams[s];
        views[s] = StreamView{d.key.p, d.fwd.p, d.psum.p, d.run_end.p, d.next_f.p, d.next_r.p, d.n, 0};
    }
    const uint64_t RS = n_regions * n_streams;
    TIRCHK(h->d_views.ensure(n_streams));
    TIRCHK(h->d_rc.ensure(n_regions));
    TIRCHK(h->d_rl.ensure(n_regions));
    TIRCHK(h->d_rr.ensure(n_regions));
    TIRCHK(h->d_rf.ensure(n_regions));
    TIRCHK(h->d_first.ensure(RS));
    TIRCHK(h->d_end.ensure(RS));
    TIRCHK(h->d_hits.ensure(RS));
    hipStream_t st = h->stream;
    TIRCHK(hipMemcpyAsync(h->d_views.p, views.data(), n_streams * sizeof(StreamView), hipMemcpyHostToDevice, st));
    TIRCHK(hipMemcpyAsync(h->d_rc.p, contig, n_regions * 4, hipMemcpyHostToDevice, st));
    TIRCHK(hipMemcpyAsync(h->d_rl.p, left, n_regions * 4, hipMemcpyHostToDevice, st));
    TIRCHK(hipMemcpyAsync(h->d_rr.p, right, n_regions * 4, hipMemcpyHostToDevice, st));
    TIRCHK(hipMemcpyAsync(h->d_rf.p, forward, n_regions, hipMemcpyHostToDevice, st));
    TIRCHK(hipEventRecord(h->ev[0], st));
    const uint64_t nb = (RS + 255) / 256;
    hipLaunchKernelGGL(tir_query, dim3((uint32_t)nb), dim3(256), 0, st, h->d_views.p, n_streams,
                       n_regions, h->d_rc.p, h->d_rl.p, h->d_rr.p, h->d_rf.p, h->d_first.p,
                       h->d_end.p, h->d_hits.p);
    TIRCHK(hipGetLastError());
    TIRCHK(hipEventRecord(h->ev[1], st));
    TIRCHK(hipMemcpyAsync(first, h->d_first.p, RS * 4, hipMemcpyDeviceToHost, st));
    TIRCHK(hipMemcpyAsync(end, h->d_end.p, RS * 4, hipMemcpyDeviceToHost, st));
    TIRCHK(hipMemcpyAsync(hits, h->d_hits.p, RS * 4, hipMemcpyDeviceToHost, st));
    TIRCHK(hipStreamSynchronize(st));
    float ms = 0;
    TIRCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->last_ms[1] = ms;
    return UP_OK;
}

int up_tir_timings(up_tir *h, double *ms, int n) {
    if (!h || !ms || n < 0) return UP_E_ARG;
    for (int i = 0; i < n && i < 2; ++i) ms[i] = h->last_ms[i];
    return UP_OK;
}

}  // extern "C"
