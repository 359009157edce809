// unipeak_amd/csrc/countmap.hip -- bin/convert_align's CountMap on the GPU
// (include/unipeak_hip.h "convert_align").
//
// The reference keeps one std::map<Pos, HitCount> per (strand, contig)
// (misc/data.cpp:263-314) and then walks them in order (ConstIterator,
// ConstNondirIterator, misc/data.cpp:321-596).  On MI355X the whole genome's
// counts fit in HBM as dense uint32 tracks, [strand][contig][position]
// (hg19: 2 x 3.1 G x 4 B = 24.8 GB of 288 GB): an add is one atomicAdd into
// its track (uint32 wrap, like HitCount), and the ordered walk is a stream
// compaction of the nonzero positions -- a count pass per 8,192-position
// block, a host scan of the block counts, and an emit pass writing the
// entries in exactly the iterators' order (position-ascending inside a
// contig, contigs in table order, forward strand before reverse; merged
// strands with summed counts for nondirectional output).  Both passes stream
// the tracks once with 16-byte loads: HBM-bound.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/unipeak_hip.h"

namespace {

constexpr int kThreads = 256;
constexpr int kIters = 8;                                 // 16-byte loads per thread per block
constexpr uint64_t kBlockPos = (uint64_t)kThreads * 4 * kIters;  // 8,192 positions

__global__ void __launch_bounds__(256) cm_add(uint32_t *__restrict__ tracks, uint64_t genome,
                                              const uint64_t *__restrict__ off,
                                              const uint32_t *__restrict__ len, uint32_t n_contigs,
                                              uint64_t n, const uint32_t *__restrict__ contig,
                                              const uint32_t *__restrict__ pos,
                                              const uint8_t *__restrict__ fwd,
                                              const uint32_t *__restrict__ cnt,
                                              uint32_t *__restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = contig[i], p = pos[i];
    if (c >= n_contigs || p == 0 || p > len[c]) {
        atomicOr(err, 1u);
        return;
    }
    const uint64_t at = (fwd[i] ? 0 : genome) + off[c] + p - 1;
    atomicAdd(&tracks[at], cnt ? cnt[i] : 1u);
}

// the value of view position v: directional = the concatenated [fwd | rev]
// tracks; nondirectional = fwd + rev at the same position (uint32 wrap)
__device__ __forceinline__ uint4 load4(const uint32_t *tracks, uint64_t genome, uint64_t view_n,
                                       int nondir, uint64_t v) {
    uint4 a = make_uint4(0, 0, 0, 0);
    if (v + 4 <= view_n && (v & 3) == 0) {
        a = *reinterpret_cast<const uint4 *>(tracks + v);
        if (nondir) {
            // the reverse half starts at `genome`: 16-byte aligned only when
            // genome % 4 == 0, else four dword loads
            const uint32_t *r = tracks + genome + v;
            uint4 b;
            if ((genome & 3) == 0) b = *reinterpret_cast<const uint4 *>(r);
            else b = make_uint4(r[0], r[1], r[2], r[3]);
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
    } else {
        uint32_t t[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k)
            if (v + k < view_n) t[k] = tracks[v + k] + (nondir ? tracks[genome + v + k] : 0u);
        a = make_uint4(t[0], t[1], t[2], t[3]);
    }
    return a;
}

__global__ void __launch_bounds__(kThreads) cm_count(const uint32_t *__restrict__ tracks,
                                                     uint64_t genome, uint64_t view_n, int nondir,
                                                     uint32_t *__restrict__ bcount) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kBlockPos;
    uint32_t nz = 0;
#pragma unroll
    for (int k = 0; k < kIters; ++k) {
        const uint64_t v = base + (uint64_t)k * kThreads * 4 + (uint64_t)threadIdx.x * 4;
        const uint4 a = load4(tracks, genome, view_n, nondir, v);
        nz += (a.x != 0) + (a.y != 0) + (a.z != 0) + (a.w != 0);
    }
    for (int o = 32; o > 0; o >>= 1) nz += (uint32_t)__shfl_xor((int)nz, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = nz;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kThreads / 64; ++w) t += s_w[w];
        bcount[blockIdx.x] = t;
    }
}

__device__ __forceinline__ uint32_t wave_excl(uint32_t v, int lane, uint32_t *total) {
    uint32_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += t;
    }
    *total = (uint32_t)__shfl((int)x, 63, 64);
    return x - v;
}

__global__ void __launch_bounds__(kThreads) cm_emit(const uint32_t *__restrict__ tracks,
                                                    uint64_t genome, uint64_t view_n, int nondir,
                                                    const uint64_t *__restrict__ boff,
                                                    const uint64_t *__restrict__ off,
                                                    uint32_t n_contigs,
                                                    uint32_t *__restrict__ o_contig,
                                                    uint32_t *__restrict__ o_pos,
                                                    uint32_t *__restrict__ o_cnt,
                                                    uint8_t *__restrict__ o_fwd) {
    __shared__ uint32_t s_w[kThreads / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kBlockPos;
    uint64_t out = boff[blockIdx.x];
    for (int k = 0; k < kIters; ++k) {
        const uint64_t v = base + (uint64_t)k * kThreads * 4 + (uint64_t)threadIdx.x * 4;
        const uint4 a = load4(tracks, genome, view_n, nondir, v);
        const uint32_t val[4] = {a.x, a.y, a.z, a.w};
        const uint32_t nz = (a.x != 0) + (a.y != 0) + (a.z != 0) + (a.w != 0);
        uint32_t wtot;
        const uint32_t wex = wave_excl(nz, lane, &wtot);
        if (lane == 0) s_w[wave] = wtot;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int w = 0; w < kThreads / 64; ++w) {
            before += w < wave ? s_w[w] : 0u;
            all += s_w[w];
        }
        __syncthreads();
        if (nz) {
            uint64_t o = out + before + wex;
            for (int j = 0; j < 4; ++j) {
                if (!val[j]) continue;
                // strand and contig of view position v + j (a group of four
                // may straddle the forward/reverse boundary: the genome
                // length need not be a multiple of 4)
                const uint64_t vj = v + j;
                const bool rev = !nondir && vj >= genome;
                const uint64_t g = rev ? vj - genome : vj;
                uint32_t lo = 0, hi = n_contigs;  // last contig with off <= g
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (off[mid] <= g) lo = mid;
                    else hi = mid;
                }
                o_contig[o] = lo;
                o_pos[o] = (uint32_t)(g - off[lo] + 1);
                o_cnt[o] = val[j];
                o_fwd[o] = rev ? 0 : 1;
                ++o;
            }
        }
        out += all;
    }
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

}  // namespace

struct up_cm {
    int dev = 0;
    hipStream_t stream = nullptr;
    uint32_t n_contigs = 0;
    uint64_t genome = 0;             // positions per strand (sum of contig lengths)
    std::vector<uint64_t> off;       // [n_contigs + 1] first position of each contig
    Dev<uint32_t> tracks;            // [2 * genome]
    Dev<uint64_t> d_off;
    Dev<uint32_t> d_len, d_err;
    Dev<uint32_t> a_contig, a_pos, a_cnt;  // add staging
    Dev<uint8_t> a_fwd;
    Dev<uint32_t> bcount;
    Dev<uint64_t> boff;
    Dev<uint32_t> o_contig, o_pos, o_cnt;
    Dev<uint8_t> o_fwd;
    double ms_add = 0, ms_collect = 0;
    hipEvent_t ev[2] = {};
};

#define CMCHK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? UP_E_NOMEM : UP_E_HIP; \
    } while (0)

extern "C" {

int up_cm_open(int hip_device, uint32_t n_contigs, const uint32_t *contig_len, up_cm **out) {
    if (!out || n_contigs == 0 || !contig_len) return UP_E_ARG;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd < 1) return UP_E_NODEV;
    if (hip_device < 0 || hip_device >= nd) return UP_E_ARG;
    up_cm *h = new up_cm;
    h->dev = hip_device;
    h->n_contigs = n_contigs;
    h->off.resize(n_contigs + 1);
    for (uint32_t c = 0; c < n_contigs; ++c) h->off[c + 1] = h->off[c] + contig_len[c];
    h->genome = h->off[n_contigs];
    auto fail = [&](int code) {
        up_cm_close(h);
        return code;
    };
    if (hipSetDevice(hip_device) != hipSuccess) return fail(UP_E_HIP);
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) return fail(UP_E_HIP);
    for (auto &e : h->ev)
        if (hipEventCreate(&e) != hipSuccess) return fail(UP_E_HIP);
    if (h->tracks.ensure(2 * h->genome + 4) != hipSuccess) return fail(UP_E_NOMEM);
    if (h->d_off.ensure(n_contigs + 1) != hipSuccess || h->d_len.ensure(n_contigs) != hipSuccess ||
        h->d_err.ensure(1) != hipSuccess)
        return fail(UP_E_NOMEM);
    if (hipMemsetAsync(h->tracks.p, 0, (2 * h->genome + 4) * sizeof(uint32_t), h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_err.p, 0, sizeof(uint32_t), h->stream) != hipSuccess ||
        hipMemcpyAsync(h->d_off.p, h->off.data(), (n_contigs + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                       h->stream) != hipSuccess ||
        hipMemcpyAsync(h->d_len.p, contig_len, n_contigs * sizeof(uint32_t), hipMemcpyHostToDevice,
                       h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess)
        return fail(UP_E_HIP);
    *out = h;
    return UP_OK;
}

void up_cm_close(up_cm *h) {
    if (!h) return;
    (void)hipSetDevice(h->dev);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto *b : {&h->tracks, &h->d_len, &h->d_err, &h->a_contig, &h->a_pos, &h->a_cnt, &h->bcount,
                    &h->o_contig, &h->o_pos, &h->o_cnt})
        b->release();
    h->d_off.release();
    h->boff.release();
    h->a_fwd.release();
    h->o_fwd.release();
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int up_cm_add(up_cm *h, uint64_t n, const uint32_t *contig, const uint32_t *pos, const uint8_t *forward,
              const uint32_t *count) {
    if (!h || (n && (!contig || !pos || !forward))) return UP_E_ARG;
    if (n == 0) return UP_OK;
    CMCHK(hipSetDevice(h->dev));
    hipStream_t st = h->stream;
    CMCHK(h->a_contig.ensure(n));
    CMCHK(h->a_pos.ensure(n));
    CMCHK(h->a_fwd.ensure(n));
    if (count) CMCHK(h->a_cnt.ensure(n));
    CMCHK(hipMemcpyAsync(h->a_contig.p, contig, n * 4, hipMemcpyHostToDevice, st));
    CMCHK(hipMemcpyAsync(h->a_pos.p, pos, n * 4, hipMemcpyHostToDevice, st));
    CMCHK(hipMemcpyAsync(h->a_fwd.p, forward, n, hipMemcpyHostToDevice, st));
    if (count) CMCHK(hipMemcpyAsync(h->a_cnt.p, count, n * 4, hipMemcpyHostToDevice, st));
    CMCHK(hipEventRecord(h->ev[0], st));
    hipLaunchKernelGGL(cm_add, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, h->tracks.p, h->genome,
                       h->d_off.p, h->d_len.p, h->n_contigs, n, h->a_contig.p, h->a_pos.p, h->a_fwd.p,
                       count ? h->a_cnt.p : nullptr, h->d_err.p);
    CMCHK(hipGetLastError());
    CMCHK(hipEventRecord(h->ev[1], st));
    uint32_t err = 0;
    CMCHK(hipMemcpyAsync(&err, h->d_err.p, 4, hipMemcpyDeviceToHost, st));
    CMCHK(hipStreamSynchronize(st));
    float ms = 0;
    CMCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->ms_add += ms;
    return err ? UP_E_ARG : UP_OK;
}

int up_cm_collect(up_cm *h, int nondir, uint64_t *n, uint32_t *contig, uint32_t *pos, uint32_t *count,
                  uint8_t *forward, uint64_t cap) {
    if (!h || !n) return UP_E_ARG;
    CMCHK(hipSetDevice(h->dev));
    hipStream_t st = h->stream;
    const uint64_t view_n = nondir ? h->genome : 2 * h->genome;
    const uint64_t nblk = (view_n + kBlockPos - 1) / kBlockPos;
    CMCHK(h->bcount.ensure(nblk + 1));
    CMCHK(h->boff.ensure(nblk + 1));
    CMCHK(hipEventRecord(h->ev[0], st));
    if (nblk)
        hipLaunchKernelGGL(cm_count, dim3((uint32_t)nblk), dim3(kThreads), 0, st, h->tracks.p, h->genome,
                           view_n, nondir ? 1 : 0, h->bcount.p);
    CMCHK(hipGetLastError());
    std::vector<uint32_t> bc(nblk);
    std::vector<uint64_t> bo(nblk + 1, 0);
    if (nblk) CMCHK(hipMemcpyAsync(bc.data(), h->bcount.p, nblk * 4, hipMemcpyDeviceToHost, st));
    CMCHK(hipStreamSynchronize(st));
    for (uint64_t b = 0; b < nblk; ++b) bo[b + 1] = bo[b] + bc[b];
    const uint64_t total = bo[nblk];
    *n = total;
    if (!contig && !pos && !count && !forward) return UP_OK;
    if (!contig || !pos || !count || !forward) return UP_E_ARG;
    if (cap < total) return UP_E_NOMEM;
    CMCHK(h->o_contig.ensure(total + 1));
    CMCHK(h->o_pos.ensure(total + 1));
    CMCHK(h->o_cnt.ensure(total + 1));
    CMCHK(h->o_fwd.ensure(total + 1));
    CMCHK(hipMemcpyAsync(h->boff.p, bo.data(), (nblk + 1) * 8, hipMemcpyHostToDevice, st));
    if (nblk)
        hipLaunchKernelGGL(cm_emit, dim3((uint32_t)nblk), dim3(kThreads), 0, st, h->tracks.p, h->genome,
                           view_n, nondir ? 1 : 0, h->boff.p, h->d_off.p, h->n_contigs, h->o_contig.p,
                           h->o_pos.p, h->o_cnt.p, h->o_fwd.p);
    CMCHK(hipGetLastError());
    CMCHK(hipEventRecord(h->ev[1], st));
    if (total) {
        CMCHK(hipMemcpyAsync(contig, h->o_contig.p, total * 4, hipMemcpyDeviceToHost, st));
        CMCHK(hipMemcpyAsync(pos, h->o_pos.p, total * 4, hipMemcpyDeviceToHost, st));
        CMCHK(hipMemcpyAsync(count, h->o_cnt.p, total * 4, hipMemcpyDeviceToHost, st));
        CMCHK(hipMemcpyAsync(forward, h->o_fwd.p, total, hipMemcpyDeviceToHost, st));
    }
    CMCHK(hipStreamSynchronize(st));
    float ms = 0;
    CMCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->ms_collect = ms;
    return UP_OK;
}

int up_cm_timings(up_cm *h, double *ms, int n) {
    if (!h || !ms || n < 0) return UP_E_ARG;
    if (n > 0) ms[0] = h->ms_add;
    if (n > 1) ms[1] = h->ms_collect;
    return UP_OK;
}

}  // extern "C"
