// unipeak_amd/csrc/kernels.hip -- gfx950 kernels of the KDE smoothing +
// enriched-region scan (reference: misc/peakcall.cpp:33-231,
// misc/kernel.cpp:12-35, misc/data.cpp:22-193).
//
// Exactness contract: every score is the FP64 left-to-right sum, over the
// hits h of the window in ascending order, of kernel[x-h+bw] * countSum[h]
// (one multiply, one add -- the order ProfileBuffer::add accumulates into
// its deque cells, peakcall.cpp:203-209).  Built with -ffp-contract=off so
// no FMA fuses the pair; zero-count positions are skipped exactly as the
// reference skips countSum == 0 adds.  The work is proportional to hits, not
// taps: a wave owns 64 consecutive positions per step and walks the hit
// bitmaps (wave ballots) of the neighbouring words in ascending order,
// broadcasting each hit's pooled count with v_readlane.
//
// Kernels
//   K1 scan_kernel     pool + KDE + threshold flags + run boundaries per strip
//   K2 finalize/scatter  strip-boundary fix-up, scan, compaction to regions
//   K3 stats_kernel    per-region peak, exptSums, kurtosis, strandCorr, filter
//   K4 shift_kernel    strandCorr(shift) table for bin/strand_shift
//   aux: scatter, synthetic input, unit last-add reduction
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/unipeak_hip.h"
#include "kernels.h"

namespace upk {

__device__ __forceinline__ double rl_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ uint32_t rl_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// bits b of a word at offset d words from the output word whose hits can
// reach some lane of the output word: 64d + b in [-bw, 63 + bw]
__device__ __forceinline__ uint64_t win_mask(int d, int bw) {
    int lo = -bw - 64 * d, hi = 63 + bw - 64 * d;
    lo = lo < 0 ? 0 : lo;
    hi = hi > 63 ? 63 : hi;
    if (lo > hi) return 0;
    const uint64_t up = hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1);
    return up & ~((1ull << lo) - 1);
}

// global-address-space views of a track (plain pointers from the unit table
// would otherwise compile to flat loads)
typedef const __attribute__((address_space(1))) uint32_t gu32;
typedef const __attribute__((address_space(1))) uint8_t gu8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
// read-only kernel inputs through the constant address space: a uniform
// index then compiles to scalar loads (s_load, lgkmcnt) instead of vector
// loads whose vmcnt waits would also wait for the streaming loads in flight
#ifdef __HIP_DEVICE_COMPILE__
#define UPK_CONST __attribute__((address_space(4)))
#else
#define UPK_CONST  // the host pass only type-checks the kernels
#endif
template <typename T>
__device__ __forceinline__ const UPK_CONST T *cptr(const T *p) {
    return (const UPK_CONST T *)p;
}

// window word storage: integer pooled counts (one non-control sample's
// count, or several samples' unscaled sum -- exact in uint32: the host runs
// POOL 1 only when the largest possible sum is below 2^32, and the reference's
// double countSum of integers is that same integer), otherwise the FP64
// pooled count (coefficients, Q5)
template <int POOL>
using WinT = typename std::conditional<POOL == 2, double, uint32_t>::type;

__device__ __forceinline__ double rl_cs(uint32_t v, int l) { return (double)rl_u(v, l); }
__device__ __forceinline__ double rl_cs(double v, int l) { return rl_d(v, l); }
__device__ __forceinline__ bool nz(uint32_t v) { return v != 0u; }
__device__ __forceinline__ bool nz(double v) { return v != 0.0; }

// ---- track access (layout in kernels.h: kTB-bit counts, kPerByte per byte) ----
__device__ __forceinline__ gu8 *track_u8(const UnitDesc &U, int S, int strand, int sample) {
    return (gu8 *)U.base + ((uint64_t)strand * S + sample) * U.stride;
}

// a track's chunk-sum plane, and the unit's pooled plane (kernels.h)
__device__ __forceinline__ gu8 *plane_u8(const UnitDesc &U, int S, int strand, int sample) {
    return (gu8 *)U.base + (uint64_t)U.nstrands * S * U.stride + ((uint64_t)strand * S + sample) * (U.stride / 4);
}
__device__ __forceinline__ gu8 *pooled_u8(const UnitDesc &U, int S) {
    return (gu8 *)U.base + (uint64_t)U.nstrands * S * U.stride / 4 * 5;
}

// byte and bit offset of field n (n = kPadPos + p - 1 for position p)
__host__ __device__ __forceinline__ int64_t fbyte(int64_t n) { return n >> kLogPerByte; }
__host__ __device__ __forceinline__ uint32_t fshift(int64_t n) {
    return (uint32_t)kTB * (uint32_t)(n & (kPerByte - 1));
}

// stored field (count, or the escape kEsc) of position p, 1-based
__device__ __forceinline__ uint32_t fld_at(gu8 *t, int64_t p) {
    const int64_t n = kPadPos + p - 1;
    return ((uint32_t)t[fbyte(n)] >> fshift(n)) & kTMask;
}

// sum of the fields of a dword (escapes count as kEsc)
__device__ __forceinline__ uint32_t fsum32(uint32_t x, uint32_t acc) {
    if constexpr (kTB == 4) {
        return __builtin_amdgcn_udot8(x, 0x11111111u, acc, false);  // v_dot8_u32_u4 x all-ones
    } else {
        // a field's value = its low bit + 2 x its high bit = (both bits) +
        // (the high bit again): two accumulating v_bcnt and one v_and
        // (the low/high split took six VALU per dword)
        // (written as asm: the compiler turns the sum into two plain v_bcnt
        // and a v_add3, four VALU)
        uint32_t r;
        asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
        asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x & 0xAAAAAAAAu), "v"(r));
        return r;
    }
}

// popcount(x) + acc in one v_bcnt (K1a's one-track bound: 2 x popcount of a
// 2-bit field >= its value unless the field is an escape)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// bits of a dword that make the screen treat a chunk as exact: any escaped
// field (2-bit: a field of 3; 4-bit: any count >= 8, the escape 15 among them)
__device__ __forceinline__ uint32_t fbig32(uint32_t x) {
    if constexpr (kTB == 4) return x & 0x88888888u;
    else return x & (x >> 1) & 0x55555555u;
}
// the same bits before the field mask, OR-accumulated into acc (one shift
// and one v_and_or_b32 per dword); mask the accumulator once with kBigMask
__device__ __forceinline__ uint32_t fbig_acc(uint32_t x, uint32_t acc) {
    if constexpr (kTB == 4) {
        return x | acc;
    } else {
        // (x & (x >> 1)) | acc in one v_bitop3 (LUT 0xEA); the compiler
        // splits it into v_and + half a v_or3
        uint32_t r;
        asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(r) : "v"(x), "v"(x >> 1), "v"(acc));
        return r;
    }
}
constexpr uint32_t kBigMask = kTB == 4 ? 0x88888888u : 0x55555555u;

// escaped count (>= kEsc): two dependent loads -- the block's escape tile
// index, then the tile's byte -- and, for a count >= 255 only, a binary
// search of the entries of the position's block (UnitDesc::ovf_off indexes
// them per kOvfBlk positions).  With 2-bit tracks every peak position holding
// three or more tags is an escape; the search alone (about six dependent
// loads) was a fifth of K1b with 8 pooled samples.
// (inline: a call needs a stack frame, i.e. scratch, in every kernel using it)
__device__ __forceinline__ uint32_t ovf_lookup(const UnitDesc &U, uint32_t track, uint32_t pos) {
    if (!U.ovf || pos - 1u >= U.len) return kEsc;
    const uint32_t nblk = ovf_nblk(U.len);
    const uint32_t ti = ((const uint32_t *)U.ovf_tidx)[(size_t)track * nblk + ((pos - 1u) >> kOvfBlkShift)];
    if (ti != kNoTile) {
        const uint32_t v = ((const uint8_t *)U.ovf_tiles)[(size_t)ti * kOvfBlk + ((pos - 1u) & (kOvfBlk - 1u))];
        if (v != 255u) return v;
    }
    const uint32_t *off = (const uint32_t *)U.ovf_off + (size_t)track * (ovf_nblk(U.len) + 1) +
                          ((pos - 1u) >> kOvfBlkShift);
    const uint64_t *e = (const uint64_t *)U.ovf;
    uint32_t lo = off[0], hi = off[1];
    const uint32_t end = hi;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t p = (uint32_t)(e[mid] >> 32);
        if (p < pos) lo = mid + 1; else hi = mid;
    }
    return (lo < end && (uint32_t)(e[lo] >> 32) == pos) ? (uint32_t)e[lo] : kEsc;
}

// escapes of N words (lane's position x0 + 64w + lane in word w): each lane
// resolves its own escaped words, one lookup per round, so the rounds are the
// most escapes any lane holds rather than the words with an escape anywhere
template <int N>
__device__ __forceinline__ void resolve_escapes(uint32_t (&c)[N], const UnitDesc &U, uint32_t track, int64_t x0,
                                                int lane) {
    uint32_t m = 0;
#pragma unroll
    for (int w = 0; w < N; ++w) m |= (c[w] == kEsc ? 1u : 0u) << w;
    while (m) {
        const int w = __builtin_ctz(m);
        m &= m - 1;
        const uint32_t v = ovf_lookup(U, track, (uint32_t)(x0 + 64 * w + lane));
#pragma unroll
        for (int q = 0; q < N; ++q) c[q] = q == w ? v : c[q];
    }
}

// exact count of (strand, sample) at position p (1-based)
__device__ __forceinline__ uint32_t count_at(const UnitDesc &U, int S, int strand, int sample,
                                             int64_t p) {
    const uint32_t b = fld_at(track_u8(U, S, strand, sample), p);
    return b == kEsc ? ovf_lookup(U, (uint32_t)(strand * S + sample), (uint32_t)p) : b;
}

// pooled counts of N words from the unit's pooled count track (POOL 1): one
// coalesced byte load per word; a saturated byte (255) is summed from the
// samples' tracks in the reference's sample order (exact in uint32)
template <int N>
__device__ __forceinline__ void pct_words(uint32_t (&c)[N], const UnitDesc &U, int S, int strand, int64_t x0,
                                          int lane, int nnc, const int32_t *nc) {
    gu8 *t = (gu8 *)U.pct + (uint64_t)strand * ((uint64_t)kPerByte * U.stride) + (kPadPos + x0 - 1 + lane);
#pragma unroll
    for (int w = 0; w < N; ++w) c[w] = t[64 * w];
    uint32_t m = 0;
#pragma unroll
    for (int w = 0; w < N; ++w) m |= (c[w] == 255u ? 1u : 0u) << w;
    while (m) {
        const int w = __builtin_ctz(m);
        m &= m - 1;
        uint32_t v = 0;
        for (int k = 0; k < nnc; ++k) v += count_at(U, S, strand, nc[k], x0 + 64 * w + lane);
#pragma unroll
        for (int q = 0; q < N; ++q) c[q] = q == w ? v : c[q];
    }
}

// ---- pooled count (ProfileBuffer::add countSum, peakcall.cpp:186-200) ----
// POOL 0: one non-control sample, no coefficients; 1: several, unscaled;
// 2: scaled by coefficients plus the unscaled second loop (quirk Q5).
// x0 = position of lane 0 of the first word.
template <int N, int POOL>
__device__ __forceinline__ void load_words(WinT<POOL> (&cs)[N], const UnitDesc &U, int S, int strand,
                                           int64_t x0, int lane, int nnc, const int32_t *nc,
                                           const double *coef) {
    uint32_t c[N];
    auto fetch = [&](int k) {
        // lane's field n0 + 64w = byte fbyte(n0) + kWordBytes * w, same bits for every w
        const int64_t n0 = kPadPos + x0 - 1 + lane;
        gu8 *t = track_u8(U, S, strand, nc[k]) + fbyte(n0);
        const uint32_t sh = fshift(n0);
#pragma unroll
        for (int w = 0; w < N; ++w) c[w] = t[kWordBytes * w];
#pragma unroll
        for (int w = 0; w < N; ++w) c[w] = (c[w] >> sh) & kTMask;
        resolve_escapes<N>(c, U, (uint32_t)(strand * S + nc[k]), x0, lane);
    };
    if constexpr (POOL == 0) {
        fetch(0);
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = c[w];
    } else if (POOL == 1 && U.pct) {
        pct_words<N>(c, U, S, strand, x0, lane, nnc, nc);
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = c[w];
    } else {
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = 0;
        for (int k = 0; k < nnc; ++k) {
            fetch(k);
            if constexpr (POOL == 1) {
#pragma unroll
                for (int w = 0; w < N; ++w) cs[w] += c[w];
            } else {
                const double q = coef[k];
#pragma unroll
                for (int w = 0; w < N; ++w) cs[w] = cs[w] + (double)c[w] * q;
            }
        }
        if constexpr (POOL == 2) {
            for (int k = 0; k < nnc; ++k) {
                fetch(k);
#pragma unroll
                for (int w = 0; w < N; ++w) cs[w] = cs[w] + (double)c[w];
            }
        }
    }
}

#ifndef UPK_KHB
#define UPK_KHB 4
#endif
constexpr int kHB = UPK_KHB;  // hits per batch in the KDE walks
// Kernel weights live in LDS with kKPad zero doubles on both sides, so every
// (lane, hit) index of a window walk is a valid read and out-of-window pairs
// add exactly +0 (accumulators start at +0 and never become -0, so x + 0 == x
// bit for bit): no compare/select per pair.
constexpr int kKPad = 64 * 3;
constexpr int kKTab = 2 * kKPad + 2 * kMaxBw + 2;  // doubles of the padded table

// fill the padded table; returns the pointer to weight 0
__device__ __forceinline__ double *load_ktab(double *lds, const double *kern, int bw) {
    for (int i = threadIdx.x; i < kKTab; i += blockDim.x) {
        const int j = i - kKPad;
        lds[i] = (j >= 0 && j <= 2 * bw) ? kern[j] : 0.0;
    }
    __syncthreads();
    return lds + kKPad;
}
constexpr int kStatCache = 16;  // K3: 64-position blocks of pass-1 totals kept in LDS
// + per wave one word's kurtosis terms, compacted (pass 2's ordered sums read
// them back with broadcast LDS loads)
#ifndef UPK_TB
#define UPK_TB 4
#endif
constexpr int kTermBatch = UPK_TB;  // pass-2 term pairs loaded per batch
constexpr size_t kStatLds = kKTab * sizeof(double) + 4 * kStatCache * 64 * sizeof(uint32_t) +
                            4 * 64 * 2 * sizeof(double);

// next batch of up to kHB set bits of m (ascending) with their broadcast counts
template <typename T>
__device__ __forceinline__ void next_hits(uint64_t &m, T v, int (&b)[kHB], double (&c)[kHB]) {
#pragma unroll
    for (int h = 0; h < kHB; ++h) {
        if (m) {
            b[h] = __builtin_ctzll(m);
            m &= m - 1;
            c[h] = rl_cs(v, b[h]);
        } else {  // unused slot: a +0 contribution from an in-range index
            b[h] = 0;
            c[h] = 0.0;
        }
    }
}

// Same as load_words, but the N*kWordBytes bytes of each track are fetched
// with 16-byte lane loads (one 1 KiB wave load per 1024/kWordBytes words) and
// turned into the lane = position layout through this wave's LDS stage
// (kStageBytes per strand).  x0 - 1 must be a multiple of 64 (the bytes are
// then 16-byte aligned).  Several pooled samples are fetched in batches: the
// lanes of one set of wave loads cover up to kStageBytes / (N*kWordBytes)
// tracks at once (lane l -> track l / NL, piece l % NL), so a batch costs one
// memory round trip instead of one per sample (hg19, 8 samples + 1 control:
// K1b load phase was 48 % of its clocks with one trip per sample).
constexpr int kStageBytes = 4096;
template <int N, int POOL>
__device__ __forceinline__ void load_words_staged(WinT<POOL> (&cs)[N], const UnitDesc &U, int S, int strand,
                                                  int64_t x0, int lane, int nnc, const int32_t *nc,
                                                  const double *coef, uint8_t *stage) {
    constexpr int NL = N * kWordBytes / 16;    // 16-byte lane loads per track
    static_assert(NL * 16 <= kStageBytes, "one track's window fits the stage");
    const uint32_t sh = fshift(lane);
    const int64_t b0 = fbyte(kPadPos + x0 - 1);
    if constexpr (POOL == 0) {
        constexpr int NV = (NL + 63) / 64;           // wave loads per track
        gu32x4 *t = (gu32x4 *)(track_u8(U, S, strand, nc[0]) + b0);
        u32x4 v[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q)
            if (64 * q + lane < NL) v[q] = t[64 * q + lane];
        __builtin_amdgcn_wave_barrier();  // earlier readers of the stage are done
        uint32_t eb = 0;  // escaped fields in this lane's 16 bytes
#pragma unroll
        for (int q = 0; q < NV; ++q)
            if (64 * q + lane < NL) {
                *(u32x4 *)(stage + 16 * (64 * q + lane)) = v[q];
                eb |= fbig32(v[q].x) | fbig32(v[q].y) | fbig32(v[q].z) | fbig32(v[q].w);
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t c[N];
#pragma unroll
        for (int w = 0; w < N; ++w) c[w] = ((uint32_t)stage[kWordBytes * w + fbyte(lane)] >> sh) & kTMask;
        // most windows hold no escape: one ballot instead of N per-word tests
        if (__ballot(eb != 0u)) resolve_escapes<N>(c, U, (uint32_t)(strand * S + nc[0]), x0, lane);
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = c[w];
    } else if (POOL == 1 && U.pct) {
        uint32_t c[N];
        pct_words<N>(c, U, S, strand, x0, lane, nnc, nc);
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = c[w];
    } else {
        // tracks per batch: two wave loads' worth (more held the K1b
        // register budget: 14 tracks in flight spilled)
        constexpr int NQ = 2;
        constexpr int KB = (NQ * 64 / NL) < (kStageBytes / (NL * 16)) ? NQ * 64 / NL : kStageBytes / (NL * 16);
#pragma unroll
        for (int w = 0; w < N; ++w) cs[w] = 0;
        // POOL 2: the coefficient-weighted loop, then the unweighted one (Q5)
        for (int pass = 0; pass < (POOL == 2 ? 2 : 1); ++pass) {
            for (int k0 = 0; k0 < nnc; k0 += KB) {
                const int kb = nnc - k0 < KB ? nnc - k0 : KB;
                u32x4 v[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int l = 64 * q + lane;
                    if (l < kb * NL) {
                        const int k = k0 + l / NL;
                        v[q] = ((gu32x4 *)(track_u8(U, S, strand, nc[k]) + b0))[l % NL];
                    }
                }
                __builtin_amdgcn_wave_barrier();  // earlier readers of the stage are done
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    if (64 * q + lane < kb * NL) *(u32x4 *)(stage + 16 * (64 * q + lane)) = v[q];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int k = 0; k < kb; ++k) {  // sample order: the reference's summation order
                    uint32_t c[N];
#pragma unroll
                    for (int w = 0; w < N; ++w)
                        c[w] = ((uint32_t)stage[NL * 16 * k + kWordBytes * w + fbyte(lane)] >> sh) & kTMask;
                    resolve_escapes<N>(c, U, (uint32_t)(strand * S + nc[k0 + k]), x0, lane);
                    if constexpr (POOL == 1) {
#pragma unroll
                        for (int w = 0; w < N; ++w) cs[w] += c[w];
                    } else if (pass == 0) {
                        const double q = coef[k0 + k];
#pragma unroll
                        for (int w = 0; w < N; ++w) cs[w] = cs[w] + (double)c[w] * q;
                    } else {
#pragma unroll
                        for (int w = 0; w < N; ++w) cs[w] = cs[w] + (double)c[w];
                    }
                }
                __builtin_amdgcn_wave_barrier();  // stage free for the next batch
            }
        }
    }
    __builtin_amdgcn_wave_barrier();  // stage free for the next fetch
}

// KDE value of lane's position in output word K: ascending walk over the
// hits of words K-NH..K+NH (window-masked).  K must be a compile-time index.
template <int NWT, int NH, int K, typename T>
__device__ __forceinline__ double kde_word(const T (&cs)[NWT], const uint64_t (&hm)[NWT],
                                           const uint64_t (&wm)[2 * NH + 1], int lane, int bw,
                                           const double *ktab) {
    double f = 0.0;
#pragma unroll
    for (int d = -NH; d <= NH; ++d) {
        uint64_t m = hm[K + d] & wm[d + NH];
        while (m) {  // batches of kHB hits: weight reads first, adds in order
            int b[kHB];
            double c[kHB], kv[kHB];
            next_hits(m, cs[K + d], b, c);
#pragma unroll
            for (int h = 0; h < kHB; ++h) kv[h] = ktab[lane + (bw - 64 * d - b[h])];  // 0 outside
#pragma unroll
            for (int h = 0; h < kHB; ++h) f = f + kv[h] * c[h];
        }
    }
    return f;
}

template <int NWT, int NH, int K>
__device__ __forceinline__ uint64_t any_hits(const uint64_t (&hm)[NWT], const uint64_t (&wm)[2 * NH + 1]) {
    uint64_t a = 0;
#pragma unroll
    for (int d = -NH; d <= NH; ++d) a |= hm[K + d] & wm[d + NH];
    return a;
}

template <int K0, int K1>
struct WordLoop {
    template <typename F>
    __device__ __forceinline__ static void run(F &&fn) {
        fn(std::integral_constant<int, K0>());
        WordLoop<K0 + 1, K1>::run(fn);
    }
};
template <int K1>
struct WordLoop<K1, K1> {
    template <typename F>
    __device__ __forceinline__ static void run(F &&) {}
};

template <typename UP>
__device__ __forceinline__ uint32_t find_unit(UP units, uint32_t nunits, uint32_t strip) {
    uint32_t lo = 0, hi = nunits;  // last unit with strip0 <= strip
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (units[mid].strip0 <= strip) lo = mid; else hi = mid;
    }
    return lo;
}

// run-boundary record list of one strip: kCap inline starts/ends, spilled
// to an overflow slot (kOvfHalf each) by lane 0 when either list fills
// run-boundary record list of one strip: kCap inline starts/ends (+ end
// peaks), spilled to an overflow slot (kOvfHalf each) by lane 0 when either
// list fills.  Index-based, so the uniform state is three scalars.
constexpr uint32_t kInline = 0xFFFFFFFFu;
struct RecList {
    uint32_t ns, ne;
    uint32_t slot;  // kInline, an overflow slot, or >= ovf_cap when lost
};

__device__ __forceinline__ uint32_t *rec_area(const ScanParams &P, const RecList &R, uint32_t strip,
                                               uint32_t &half) {
    if (R.slot == kInline) {
        half = kCap;
        return P.rec + (uint64_t)strip * kRecStride;
    }
    half = kOvfHalf;
    return P.ovf_rec + (uint64_t)R.slot * kOvfStride;
}

__device__ __forceinline__ void rec_spill(RecList &R, const ScanParams &P, uint32_t strip, int lane) {
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(P.ovf_count, 1u);
    slot = rl_u(slot, 0);
    uint32_t *inl = P.rec + (uint64_t)strip * kRecStride;
    if (slot < P.ovf_cap && lane == 0) {  // same lane wrote the inline records: program order suffices
        uint32_t *dst = P.ovf_rec + (uint64_t)slot * kOvfStride;
        for (uint32_t i = 0; i < R.ns; ++i) dst[i] = inl[i];
        for (uint32_t i = 0; i < R.ne; ++i) {
            dst[kOvfHalf + i] = inl[kCap + i];
            dst[2 * kOvfHalf + i] = inl[2 * kCap + i];
            ((double *)(dst + 4 * kOvfHalf))[i] = ((const double *)(inl + 4 * kCap))[i];
        }
    }
    if (lane == 0) inl[0] = slot;  // compact reads the slot here (>= ovf_cap: host reruns)
    R.slot = slot;
}

__device__ __forceinline__ void rec_start(RecList &R, uint32_t pos, const ScanParams &P, uint32_t strip,
                                          int lane) {
    if (R.slot == kInline && R.ns == kCap) rec_spill(R, P, strip, lane);
    if (lane == 0 && (R.slot == kInline || R.slot < P.ovf_cap)) {
        uint32_t half;
        rec_area(P, R, strip, half)[R.ns] = pos;
    }
    ++R.ns;
}

__device__ __forceinline__ void rec_end(RecList &R, uint32_t pos, uint32_t pk_pos, double pk_val,
                                        const ScanParams &P, uint32_t strip, int lane) {
    if (R.slot == kInline && R.ne == kCap) rec_spill(R, P, strip, lane);
    if (lane == 0 && (R.slot == kInline || R.slot < P.ovf_cap)) {
        uint32_t half;
        uint32_t *a = rec_area(P, R, strip, half);
        a[half + R.ne] = pos;
        a[2 * half + R.ne] = pk_pos;
        ((double *)(a + 4 * half))[R.ne] = pk_val;
    }
    ++R.ne;
}

// Wave reductions through DPP (VALU only; a __shfl_xor step is an LDS
// bpermute plus its address arithmetic): row_shr 1, 2, 4, 8 leave each
// 16-lane row's total in its lane 15, row_bcast 15 / 31 carry rows 0-1 and
// 0-2 into rows 1 and 2-3, lane 63 ends with the wave's total, read back as
// a wave-uniform value.  The ops are associative and commutative (u32 wrap
// sums, min, max of non-NaN), so the result equals the butterfly's.  `id` is
// the identity that lanes without a source keep.  Every lane must be active.
template <int CTRL, int ROWS, bool ZERO>
__device__ __forceinline__ uint32_t dpp32(uint32_t id, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, ROWS, 0xf, ZERO);
}
template <typename Op>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v, uint32_t id, Op op) {
    v = op(v, dpp32<0x111, 0xf, false>(id, v));
    v = op(v, dpp32<0x112, 0xf, false>(id, v));
    v = op(v, dpp32<0x114, 0xf, false>(id, v));
    v = op(v, dpp32<0x118, 0xf, false>(id, v));
    v = op(v, dpp32<0x142, 0xa, false>(id, v));
    v = op(v, dpp32<0x143, 0xc, false>(id, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp64(double id, double v) {
    const uint64_t a = (uint64_t)__double_as_longlong(id), b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = dpp32<CTRL, ROWS, false>((uint32_t)a, (uint32_t)b);
    const uint32_t hi = dpp32<CTRL, ROWS, false>((uint32_t)(a >> 32), (uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return wave_reduce_u32(v, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return b < a ? b : a; });
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return b > a ? b : a; });
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return wave_reduce_u32(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}

// inclusive wave prefix sum (u32, wrapping): the same DPP steps, each lane
// adding the partial of the lane n below it (row_shr, 0 past the row start),
// then the row totals carried by row_bcast 15 / 31
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v) {
    v += dpp32<0x111, 0xf, true>(0u, v);
    v += dpp32<0x112, 0xf, true>(0u, v);
    v += dpp32<0x114, 0xf, true>(0u, v);
    v += dpp32<0x118, 0xf, true>(0u, v);
    v += dpp32<0x142, 0xa, false>(0u, v);
    v += dpp32<0x143, 0xc, false>(0u, v);
    return v;
}

__device__ __forceinline__ double wave_max_d(double v) {
    const double ninf = -__builtin_inf();
    v = __builtin_fmax(v, dpp64<0x111, 0xf>(ninf, v));
    v = __builtin_fmax(v, dpp64<0x112, 0xf>(ninf, v));
    v = __builtin_fmax(v, dpp64<0x114, 0xf>(ninf, v));
    v = __builtin_fmax(v, dpp64<0x118, 0xf>(ninf, v));
    v = __builtin_fmax(v, dpp64<0x142, 0xa>(ninf, v));
    v = __builtin_fmax(v, dpp64<0x143, 0xc>(ninf, v));
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// scatter up to kHB hits (window word W, bits b[], pooled counts c[], in
// ascending order; c = 0 marks an unused slot) into the register
// accumulators of the live output words they reach.  The kernel-weight reads
// of the whole batch are issued before the first add, so the LDS latency is
// paid once per batch rather than once per hit; the adds stay in hit order
// (mul, then add: the reference's accumulation, peakcall.cpp:203-209).
template <int NH, int SW, int W, typename A>
__device__ __forceinline__ void scatter_hits(A (&acc)[SW], const int (&b)[kHB], const double (&c)[kHB],
                                             int lane, int bw, const double *ktab, uint32_t live) {
    // Every weight read of the batch -- all output words in reach, live or
    // not (the padded table keeps every index valid) -- is issued before the
    // first multiply, so one LDS latency is paid per batch instead of one per
    // output word; the volatile view keeps the compiler from sinking a read
    // into its word's live branch.
    constexpr int T0 = W - NH < NH ? NH : W - NH;           // first output window word in reach
    constexpr int T1 = W + NH > NH + SW - 1 ? NH + SW - 1 : W + NH;
    constexpr int NT = T1 - T0 + 1;
    typedef const volatile __attribute__((address_space(3))) double lds_vd;
    lds_vd *vk = (lds_vd *)ktab;
    double kv[NT > 0 ? NT : 1][kHB];
    int base[kHB];
#pragma unroll
    for (int h = 0; h < kHB; ++h) base[h] = lane + bw - b[h];
#pragma unroll
    for (int q = 0; q < NT; ++q) {
#pragma unroll
        for (int h = 0; h < kHB; ++h) kv[q][h] = vk[base[h] + 64 * (T0 + q - W)];  // 0 outside
    }
    WordLoop<0, (NT > 0 ? NT : 0)>::run([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int t = T0 + q;
        if (!((live >> (t - NH)) & 1u)) return;  // uniform: word holds no flag
        // output word t-NH, lane position 64(t-NH)+lane; hit at 64(W-NH)+b
#pragma unroll
        for (int h = 0; h < kHB; ++h) acc[t - NH] = acc[t - NH] + kv[q][h] * c[h];
    });
}

// ------------------------------------------------------------------------
// K1: one wave owns one 16384-position strip of a unit (16 blocks of 1024).
//
// Screen (integer, HBM-streaming): the strip's uint8 counts of every pooled
// track are read once with 16-byte lane loads (one 1 KiB wave load per
// block), reduced to per-16-position chunk sums (v_sad_u8), and every chunk's
// window of +-R = ceil(bw/16) chunks is summed.  kmax * (weighted window
// sum) bounds every score in the chunk, so a block whose chunks all stay
// <= wskip holds no flagged position and is skipped -- no FP64 work at all.
// Exact blocks (peaks, and any chunk with a byte >= 128 / escape) run the
// KDE: the hits of the block's 16 + 2*NH words (64 positions each, re-read
// from L2 as lane = position) are walked in ascending order with wave
// ballots and scattered into FP64 accumulators, so every position's sum
// keeps the reference's order; flags give run boundaries.
// ------------------------------------------------------------------------
// chunk sums of one strip + halos, one pad word after every 16: chunk index
// i lives at word i + i/16, so the reads below (lane l takes indices 16l ..
// 16l + 31, the same offset on every lane) hit 64 different banks; unpadded,
// that 16-word lane stride made every read a 16-way bank conflict
constexpr int kScrIdx = kScrHalo + kBlocks * kWave + kScrHalo;
constexpr int kScrWords = kScrIdx + kScrIdx / 16 + 2;  // even: 8-byte aligned per wave
__device__ __forceinline__ int scr_at(int i) { return i + (i >> 4); }
// K1a needs no kernel weights: its chunk-sum areas start at LDS offset 0, so
// the lane reads of the screen fold into the ds_read2 offset fields
constexpr size_t kScreenLds = 4 * kScrWords * sizeof(uint32_t);
constexpr size_t kScanLds = kKTab * sizeof(double) + kScreenLds + 4 * kStepWords * kWave * sizeof(double);
constexpr int kXFront = 2;  // K1b work items with >= this many exact blocks go first
constexpr size_t kExactLds = kKTab * sizeof(double) + 4 * kStepWords * kWave * sizeof(double);
static_assert(2 * kStageBytes <= kStepWords * kWave * sizeof(double), "both strands' stages fit a wave's score area");

// chunks 16l .. 16l+15 of lane l that can hold a position with score >= thr.
// rd = this lane's row of the padded chunk-sum area (index 16l + j, j =
// 0..31, holds chunk 16l + j - 8).  Two bounds, both upper bounds of every
// score in the chunk:
//  * coarse (integer): kmax * (tags of the lane's span [16l - R, 16l+15+R]);
//    most lanes hold a handful of background tags, and when no lane's span
//    exceeds wskip the wave is done (wave-uniform);
//  * fine (FP32, distance-aware): sum over d of fw[|d|] * (tags of chunk
//    c + d), fw[d] = the largest kernel weight at the smallest distance
//    between positions of chunks d apart, inflated by 1e-4 (far above the
//    FP32 rounding of <= 9 positive terms).  Tags two or more chunks away
//    weigh less than kmax, so peak flanks stop failing the screen.
template <int R>
__device__ __forceinline__ uint32_t screen_bits(const uint32_t *rd, uint32_t wskip, const float *fw, float fthr) {
    uint32_t a[16 + 2 * R];  // chunks 16l - R .. 16l + 15 + R
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < 16 + 2 * R; ++j) {
        const int i = kScrHalo - R + j;
        a[j] = rd[i + (i >> 4)];
    }
#pragma unroll
    for (int j = 0; j < 16 + 2 * R; ++j) tot += a[j];
    if (__ballot(tot > wskip) == 0) return 0u;
    float f[16 + 2 * R];
#pragma unroll
    for (int j = 0; j < 16 + 2 * R; ++j) f[j] = (float)a[j];  // exact: sums < 2^24
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float b = fw[0] * f[i + R];
#pragma unroll
        for (int d = 1; d <= R; ++d) b = __builtin_fmaf(fw[d], f[i + R - d] + f[i + R + d], b);
        m |= (b > fthr ? 1u : 0u) << i;
    }
    return m;
}

// screen_bits for the runtime R = ceil(bw / 16) <= RM (RM = 4 NH: only the
// windows this NH can have are instantiated, which keeps the K1a register
// count of the narrow kernels down)
template <int RM>
__device__ __forceinline__ uint32_t screen_any(int R, const uint32_t *rd, uint32_t wskip, const float *fw,
                                               float fthr) {
    if constexpr (RM > 1) {
        if (R < RM) return screen_any<RM - 1>(R, rd, wskip, fw, fthr);
    }
    return screen_bits<RM>(rd, wskip, fw, fthr);
}

// Register pre-screen over a strip's chunk sums (K1a plane path): lane l
// holds chunks 16l .. 16l+15 (a); the window of chunk c is c-R .. c+R, R <=
// 16, so it reaches the neighbouring lanes' chunks only (DPP wave shifts;
// lane 0 / 63 take the strip's halo chunks from lanes 0 / 1's hv).  The
// strip is clean when no chunk's window holds more than wskip tags -- every
// window sum exactly, as screen_bits' coarse test bounds a lane's whole span.
template <int R>
__device__ __forceinline__ bool plane_clean(const uint32_t (&a)[16], const u32x4 &hv, int lane, uint32_t wskip) {
    const uint32_t hd[4] = {hv.x, hv.y, hv.z, hv.w};
    auto hbyte = [&](int i) { return (hd[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
    uint32_t e[16 + 2 * R];  // chunks 16l - R .. 16l + 15 + R
#pragma unroll
    for (int x = 0; x < R; ++x) {
        const uint32_t lh = rl_u(hbyte(16 - R + x), 0), rh = rl_u(hbyte(x), 1);
        const uint32_t l = dpp32<0x138, 0xf, false>(0u, a[16 - R + x]);  // wave_shr:1 -> lane - 1
        const uint32_t r = dpp32<0x130, 0xf, false>(0u, a[x]);           // wave_shl:1 -> lane + 1
        e[x] = lane == 0 ? lh : l;
        e[16 + R + x] = lane == 63 ? rh : r;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) e[R + i] = a[i];
    if (wskip >= 255u) {  // a saturated chunk could hide more than wskip tags
#pragma unroll
        for (int i = 0; i < 16 + 2 * R; ++i) e[i] = e[i] == 255u ? kBig : e[i];
    }
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i <= 2 * R; ++i) w += e[i];
    uint32_t mx = w;
#pragma unroll
    for (int i = 1; i < 16; ++i) {
        w += e[i + 2 * R] - e[i - 1];
        mx = w > mx ? w : mx;
    }
    return __ballot(mx > wskip) == 0;
}
template <int RM>
__device__ __forceinline__ bool plane_clean_any(int R, const uint32_t (&a)[16], const u32x4 &hv, int lane,
                                                uint32_t wskip) {
    if constexpr (RM > 1) {
        if (R < RM) return plane_clean_any<RM - 1>(R, a, hv, lane, wskip);
    }
    return plane_clean<RM>(a, hv, lane, wskip);
}

// MODE kModeScreen (K1a): stream + screen every strip; strips without exact
// blocks get their (empty) summary, the others go to the work list.
// MODE kModeExact (K1b): run the exact blocks of the listed strips, so the
// latency-bound KDE never stalls the streaming waves.  kModeFused: both in
// one pass (the PROF profile variant, every block exact).
// K1b runs 3 waves per SIMD (168 VGPRs, a few spilled).  Alone, 4 waves
// (128 VGPRs) finish it sooner (hg19 0.28 vs 0.31 ms), but K1b runs beside
// the next passes' K1a, and fewer latency-bound K1b waves leave K1a more of
// the CU: overlapped K1a 0.72 -> 0.67 ms, bench 4,010 -> 4,160 Gbp/s;
// nondirectional 2,710 -> 2,880; 8 samples 523 -> 528 (tools/ab_libs2.sh).
// K1a keeps the compiler's choice.
#ifndef UPK_K1A_WPE
#define UPK_K1A_WPE 1
#endif
// Round 6: directional K1b at 4 waves per SIMD (<= 128 VGPRs; one pooled
// sample: 7 spilled VGPRs, several: none) -- the cold pass's K1a holds 120
// VGPRs, so three K1a waves left no room for a 168-VGPR K1b wave on their
// SIMD; same box, three alternating rounds of the cold configs[1] leg:
// 6,919 / 6,957 / 6,922 -> 7,219 / 7,170 / 7,193 Gbp/s (profiles/r06/ab_k1b4.txt).
// Nondirectional K1b stays at 3 (29-61 spilled VGPRs at 128).
#ifndef UPK_K1B_WPE
#define UPK_K1B_WPE 4
#endif
#ifndef UPK_K1B_WPE_ND
#define UPK_K1B_WPE_ND 3
#endif
#ifndef UPK_SCAN_ATTR
#define UPK_SCAN_ATTR                                                                                   \
    __attribute__((amdgpu_waves_per_eu(MODE == kModeExact ? (NONDIR ? UPK_K1B_WPE_ND : UPK_K1B_WPE) \
                                       : (MODE == kModeScreen || MODE == kModeScreenF) ? UPK_K1A_WPE \
                                                                                       : 1)))
#endif
template <int NH, int POOL, bool NONDIR, bool PROF, int MODE>
__global__ void __launch_bounds__(256) UPK_SCAN_ATTR scan_kernel(ScanParams P, uint32_t strip_begin,
                                                   uint32_t strip_end) {
    extern __shared__ double lds_[];
    // K1a, over the chunk-sum plane (kModeScreen, bw <= 255) or the 2-bit fields
    constexpr bool kScr = MODE == kModeScreen || MODE == kModeScreenF;
    const int bw = P.bw;
    double *ktab = lds_ + kKPad;
    if constexpr (!kScr) ktab = load_ktab(lds_, P.kern, bw);
    uint32_t *scr = (uint32_t *)(kScr ? lds_ : lds_ + kKTab) + (threadIdx.x >> 6) * kScrWords;
    // this wave's block scores (K1b has no screen area)
    double *scs = (MODE == kModeExact ? lds_ + kKTab : (double *)((uint32_t *)(lds_ + kKTab) + 4 * kScrWords)) +
                  (threadIdx.x >> 6) * (kStepWords * kWave);

    constexpr int SW = kStepWords;
    constexpr int NWIN = SW + 2 * NH;
    using T = WinT<POOL>;
    const auto *units = cptr(P.units);
    const auto *ncs = cptr(P.nc);
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells the compiler, so the
    // strip / unit / work-list indices derived from it live in SGPRs and the
    // unit table is read with scalar loads (vector loads of it cost a
    // dependent round trip behind the streaming loads on every strip)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const int R = (bw + kChunk - 1) / kChunk;
    const int S = P.S;
    // K1b keys (ScanParams::qmode): integer pooled counts only (no -z)
    // (several pooled samples only with -D, where K3 runs its own KDE:
    // api.hip q_mode)
    constexpr bool kQ = MODE == kModeExact && !PROF && (POOL == 0 || (POOL == 1 && NONDIR));
    const bool qm = kQ && P.qmode != 0;
    const double kthr = qm ? 0.5 : P.thr;  // a flagged position's key is >= 1
    const uint32_t bw2 = (uint32_t)(bw * bw);
    // Q's window sums read prefix sums bw positions up and bw + 1 down, i.e.
    // lanes rotated by bw (mod 64) from one of two words.  The rotation is
    // one ds_bpermute, so each source lane picks the word its unique reader
    // needs: hi side words 2NH-1 / 2NH after the output word's first window
    // word, lo side words 0 / 1 (bw >> 6 == NH - 1 for every bw of this NH).
    const int hadr = 4 * ((lane + bw) & 63), ladr = 4 * ((lane - bw - 1) & 63);
    const bool hsel = ((((lane - bw) & 63) + bw - 64 * (NH - 1)) >> 6) != 0;
    const bool lsel = ((((lane + bw + 1) & 63) - bw - 1 + 64 * NH) >> 6) != 0;
    // halo words only matter where they reach an output word
    uint64_t edge_lo[NH], edge_hi[NH];
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        edge_lo[i] = win_mask(i - NH, bw);  // window word i vs output word 0
        edge_hi[i] = win_mask(i + 1, bw);   // window word NH+SW+i vs output word SW-1
    }

    uint32_t cur = 0;
    bool have = false;
    constexpr int kLoads = kStripBytes / (kWave * 16);  // K1a wave loads per strip and track
    // K1b: multi-block entries are listed first, single-block ones after
    // them, so the first resident waves take the long items
    const uint32_t nfront = MODE == kModeExact ? P.xcount[0] : 0u;
    const uint32_t nback = MODE == kModeExact ? P.xcount[1] : 0u;
    uint32_t it_end = MODE == kModeExact ? nfront + nback : strip_end;
    uint32_t xnf = 0, xnb = 0;  // K1a: entries this wave stashed (front / back)
    uint32_t it0 = (MODE == kModeExact ? 0u : strip_begin) + wave, istep = nwaves;
#ifdef UPK_DEBUG_TIMES
    // K1b phase clocks of this wave (s_memtime), added up once at the end
    uint64_t dt_item = 0, dt_load = 0, dt_scat = 0, dt_flag = 0, n_items = 0, dt_q = 0;
#endif
    // K1a software pipeline: the loads of this wave's next (strip, track) --
    // strips it0, it0 + istep, ...; tracks (strand, pooled sample) in order --
    // are issued before the current one is reduced, so two tracks' bytes are
    // in flight per wave instead of one (the stream is latency-bound at the
    // two waves per SIMD K1a keeps, launch_scan)
    constexpr bool kPf = true;
    constexpr int SH = scr_halo(NH);  // screen halo chunks this width loads on each side
    constexpr int HL_ = SH * kChunkBytes / 16;  // halo lane loads per side (SH chunks)
    // One directional track (configs[1]): the strip's escape bit
    // (ScanParams::esc, its word loaded with the prefetch) replaces the
    // per-dword escape test (two VALU per dword) when it is clear; the exact
    // chunk sums stay (the pre-screen needs them: configs[1]'s wskip is ~4
    // tags).  (Round 4 measured a first pre-screen on 2 x popcount of each
    // dword, one v_bcnt per dword: it fails on most strips at configs[1]'s
    // threshold and then costs both.)
    // One directional track and a window that reaches at most the
    // neighbouring lanes' chunks (R <= 16, NH <= 4): K1a streams the track's
    // chunk-sum plane (kernels.h: one byte per 16 positions, escapes at their
    // counts) instead of its 2-bit fields -- a quarter of the bytes, no
    // per-dword sums and no escape tests
    constexpr bool kPlane = MODE == kModeScreen && !PROF && kTB == 2 && NH <= 4;
    constexpr bool kPooledPlane = NONDIR || POOL != 0;  // several tracks: the unit's pooled plane
    // Plane path: each wave screens a run of consecutive strips -- they
    // share a unit, so the next strips' plane addresses follow from a cursor
    // without unit-table loads -- with the next two strips' loads in flight
    uint32_t c_u = 0, c_s0 = 0, c_end = 0;     // unit of the strip being screened
    uint32_t pc_u = 0, pc_s0 = 0, pc_end = 0;  // unit of the strip being prefetched
    gu8 *pc_base = nullptr;
    u32x4 phv2 = {0u, 0u, 0u, 0u};
    if constexpr (kPlane) {
        const uint32_t nsr = strip_end - strip_begin;
        const uint32_t per = (nsr + nwaves - 1) / nwaves;
        const uint32_t off = (uint64_t)wave * per < nsr ? wave * per : nsr;
        it0 = strip_begin + off;
        it_end = it0 + per < strip_end ? it0 + per : strip_end;
        istep = 1;
    }
    auto pf_plane = [&](uint32_t strip_n, u32x4 &dv, u32x4 &dh) {
        while (strip_n >= pc_end) {  // the strip's unit (first call: search)
            pc_u = pc_end == 0 ? find_unit(units, P.nunits, strip_n) : pc_u + 1;
            const UnitDesc Un = units[pc_u];
            pc_s0 = Un.strip0;
            pc_end = Un.strip0 + Un.nstrips;
            pc_base = (kPooledPlane ? pooled_u8(Un, S) : plane_u8(Un, S, 0, ncs[0])) + kPlanePad;
        }
        gu32x4 *pl = (gu32x4 *)(pc_base + (uint64_t)(strip_n - pc_s0) * kPlaneStrip);
        dv = __builtin_nontemporal_load(pl + lane);  // 16 chunk sums per lane
        dh = u32x4{0u, 0u, 0u, 0u};
        if (lane < 2) dh = pl[lane == 0 ? -1 : kPlaneStrip / 16];  // the halos' 16 chunks each side
    };
    constexpr bool kCheap = kScr && !PROF && POOL == 0 && !NONDIR && kTB == 2 && kPf && !kPlane;
    u32x4 pv[kScr && !PROF ? kLoads : 1];
    u32x4 phv = {0u, 0u, 0u, 0u};
    uint32_t pf_strip = 0, pf_cur = 0;
    int pf_st = 0, pf_k = 0;
    bool pf_ok = false;
    // kCheap: the prefetched strip's word of the escape bitmap and its bit
    // (the bit is taken when the strip is screened, so the scalar load's
    // wait lands a strip later)
    uint32_t pf_escw = ~0u, pf_escb = 0;
    auto pf_issue = [&](uint32_t strip_n, uint32_t cur_n, int st, int k) {
        const UnitDesc Un = units[cur_n];
        const int64_t q0 = 1 + (int64_t)(strip_n - Un.strip0) * kStrip;
        gu32x4 *t = (gu32x4 *)(track_u8(Un, S, st, ncs[k]) + fbyte(kPadPos + q0 - 1));
#pragma unroll
        for (int q = 0; q < (kScr && !PROF ? kLoads : 1); ++q)
            pv[q] = __builtin_nontemporal_load(t + 64 * q + lane);
        phv = u32x4{0u, 0u, 0u, 0u};
        if (lane < 2 * HL_) phv = t[lane < HL_ ? lane - HL_ : kLoads * kWave + lane - HL_];
        if constexpr (kCheap) {
            const uint32_t *eb = cptr(P.esc);
            pf_escw = eb ? eb[(size_t)(st * S + ncs[k]) * P.esc_nw + (strip_n >> 5)] : ~0u;
            pf_escb = strip_n & 31u;
        }
        pf_strip = strip_n;
        pf_cur = cur_n;
        pf_st = st;
        pf_k = k;
        pf_ok = true;
    };
    if constexpr (kPlane) {
        if (it0 < it_end) pf_plane(it0, pv[0], phv);
        if (it0 + 1 < it_end) pf_plane(it0 + 1, pv[1], phv2);
    } else if constexpr (kScr && !PROF && kPf) {
        if (it0 < it_end) pf_issue(it0, find_unit(units, P.nunits, it0), 0, 0);
    }
    for (uint32_t it = it0; it < it_end; it += istep) {
        const uint32_t item = it;
#ifdef UPK_DEBUG_TIMES
        const uint64_t t_it0 = __builtin_amdgcn_s_memtime();
        ++n_items;
#endif
        uint32_t strip = it;
        // this lane's failing-chunk bits (chunks 16l..16l+15 = words 4l..4l+3
        // of the strip); the live words of an exact block are gathered from
        // them with four ballots when that block runs
        uint32_t mchunk = 0xFFFFu;
        uint32_t exact_blocks = 0xFFFFu;
        if constexpr (MODE == kModeExact) {
            const uint32_t ei = cptr(P.xref)[item];
            const uint32_t *e = P.xlist + (uint64_t)ei * kXEntry;
            const auto *es = cptr(e);  // the uniform words through scalar loads
            strip = es[0];
            const uint32_t e1 = es[1];
            exact_blocks = e1 & 0xFFFFu;
            mchunk = (e[2 + (lane >> 1)] >> (16 * (lane & 1))) & 0xFFFFu;
            // K1a stored the unit with the entry (no dependent binary search)
            cur = e1 >> 16;
#ifdef UPK_DEBUG_COUNTS
            if (lane == 0) atomicAdd(&P.dbg[8 + __builtin_popcount(exact_blocks)], 1ull);  // blocks per item
#endif
            if (cur == 0xFFFFu) cur = find_unit(units, P.nunits, strip);
        } else if constexpr (kPlane) {
            while (strip >= c_end) {
                c_u = c_end == 0 ? find_unit(units, P.nunits, strip) : c_u + 1;
                c_s0 = units[c_u].strip0;
                c_end = c_s0 + units[c_u].nstrips;
            }
            cur = c_u;
        } else {
            if (!have) { cur = find_unit(units, P.nunits, strip); have = true; }
            while (strip >= units[cur].strip0 + units[cur].nstrips) ++cur;
        }
        const UnitDesc U = kPlane ? UnitDesc{} : (UnitDesc)units[cur];
        const uint32_t local = kPlane ? strip - c_s0 : strip - U.strip0;
        const uint32_t unstrips = kPlane ? c_end - c_s0 : U.nstrips;
        const int64_t p0 = 1 + (int64_t)local * kStrip;  // first position of the strip

        // ---- screen: which blocks can hold a flagged position ----
        if constexpr (kPlane) {
            const u32x4 v = pv[0], hv = phv;
            pv[0] = pv[1];
            phv = phv2;
            if (it + 2 < it_end) pf_plane(it + 2, pv[1], phv2);
            // chunks 16l .. 16l+15 of lane l (a 255: >= 255 tags, unbounded)
            uint32_t a[16];
            {
                const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int i = 0; i < 16; ++i) a[i] = (d[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            }
            const bool clean = plane_clean_any<4 * NH>(R, a, hv, lane, P.wskip);
            mchunk = 0;
            exact_blocks = 0;
            if (!clean) {
                // the LDS screen of the 2-bit path over these sums: lane l's
                // chunks, the halos' 16 chunks each side from lanes 0 and 1
                uint32_t *d = scr + scr_at(kScrHalo + 16 * lane);
#pragma unroll
                for (int i = 0; i < 16; ++i) d[i] = a[i] == 255u ? kBig : a[i];
                if (lane < 2) {
                    const uint32_t hd[4] = {hv.x, hv.y, hv.z, hv.w};
                    uint32_t *h = scr + scr_at(lane == 0 ? kScrHalo - 16 : kScrHalo + kBlocks * kWave);
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t b = (hd[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                        h[i] = b == 255u ? kBig : b;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t *rd = scr + 17 * lane;  // index 16l + j = word 17l + j + j/16
                const uint32_t m = screen_any<4 * NH>(R, rd, P.wskip, P.fw, P.fthr);
                const uint64_t lanes = __ballot(m != 0u);
                mchunk = m;
#pragma unroll
                for (int bk = 0; bk < kBlocks; ++bk)
                    exact_blocks |= ((lanes >> (4 * bk)) & 0xFull) ? (1u << bk) : 0u;
                __builtin_amdgcn_wave_barrier();  // the next strip reuses scr after every lane read it
            }
        } else if constexpr (!PROF && MODE != kModeExact) {
            // lane l of wave load q holds 16 bytes = CPL chunks: chunks
            // CPL * (64q + l) + i, i < CPL (DPC dwords each)
            constexpr int CPL = 16 / kChunkBytes, DPC = kChunkBytes / 4;
            constexpr int HL = SH * kChunkBytes / 16;  // halo lane loads per side (SH chunks)
            uint32_t cs[CPL * kLoads];
            uint32_t big = 0, hs[CPL], hbig = 0;
            bool any_esc = false;  // wave-uniform: some track may hold an escape (esc_tracks)
            // tracks (strand * nnc + k < 64) whose bytes in this strip hold an
            // escape; esc_far: one of the tracks beyond the first 64 does
            uint64_t esc_tracks = 0;
            bool esc_far = false;
#pragma unroll
            for (int k = 0; k < CPL * kLoads; ++k) cs[k] = 0;
#pragma unroll
            for (int i = 0; i < CPL; ++i) hs[i] = 0;
            bool clean = false;
            bool pre_done = false;  // kCheap's packed pre-screen ran (and failed)
            // the pre-screen bound of every lane: max over its groups of the
            // tags of groups g-D .. g+D, plus both halos (below)
            auto pre_bound = [&](const uint32_t (&T)[kLoads], uint32_t hl) -> uint32_t {
                const int D = (R + CPL - 1) / CPL;
                uint32_t htot = 0;  // both halos (lanes 0 .. 2HL-1)
#pragma unroll
                for (int l = 0; l < 2 * HL; ++l) htot += rl_u(hl, l);
                uint32_t l1[kLoads], r1[kLoads], bmax = 0;
#pragma unroll
                for (int q = 0; q < kLoads; ++q) {
                    l1[q] = dpp32<0x138, 0xf, false>(0u, T[q]);  // wave_shr:1 -> T(g - 1)
                    r1[q] = dpp32<0x130, 0xf, false>(0u, T[q]);  // wave_shl:1 -> T(g + 1)
                    const uint32_t lf = q > 0 ? rl_u(T[q > 0 ? q - 1 : 0], 63) : 0u;
                    const uint32_t rf = q + 1 < kLoads ? rl_u(T[q + 1 < kLoads ? q + 1 : q], 0) : 0u;
                    l1[q] = lane == 0 ? lf : l1[q];
                    r1[q] = lane == 63 ? rf : r1[q];
                }
#pragma unroll
                for (int q = 0; q < kLoads; ++q) {
                    uint32_t b = T[q] + l1[q] + r1[q];
                    if (D == 2) {
                        uint32_t l2 = dpp32<0x138, 0xf, false>(0u, l1[q]);  // T(g - 2)
                        uint32_t r2 = dpp32<0x130, 0xf, false>(0u, r1[q]);  // T(g + 2)
                        const uint32_t lf = q > 0 ? rl_u(l1[q > 0 ? q - 1 : 0], 63) : 0u;
                        const uint32_t rf = q + 1 < kLoads ? rl_u(r1[q + 1 < kLoads ? q + 1 : q], 0) : 0u;
                        l2 = lane == 0 ? lf : l2;
                        r2 = lane == 63 ? rf : r2;
                        b += l2 + r2;
                    }
                    bmax = b > bmax ? b : bmax;
                }
                return bmax + htot;
            };
            if constexpr (kCheap) {
                u32x4 v[kLoads];
#pragma unroll
                for (int q = 0; q < kLoads; ++q) v[q] = pv[q];
                const u32x4 hv = phv;
                const bool mesc = (pf_escw >> pf_escb) & 1u;
                pf_ok = false;
                if (it + istep < it_end) {
                    uint32_t nc_ = cur;
                    while (it + istep >= units[nc_].strip0 + units[nc_].nstrips) ++nc_;
                    pf_issue(it + istep, nc_, 0, 0);
                }
                // Packed pre-screen (R <= CPL: a position's window lies in its
                // 64-position group g and the groups beside it; no escape in
                // reach, so the fields are the counts): the group sums of the
                // lane's four loads, capped at 31, as the bytes of one dword;
                // one DPP rotate each way brings the neighbouring lanes' groups
                // (lane 0 / 63: the other end of the wave shifted by a byte,
                // plus the halo group beside the strip), one 32-bit add sums
                // all four triples (<= 93 per byte, no carry), and a bytewise
                // compare against wskip + 1 < 32 settles the strip -- about
                // half the VALU of the chunk sums + per-load DPP bound below,
                // which then run only for strips that fail here.
                if (R <= CPL && P.wskip < 31u && !mesc) {
                    pre_done = true;
                    uint32_t pk = 0;
#pragma unroll
                    for (int q = 0; q < kLoads; ++q) {
                        uint32_t t = fsum32(v[q].x, 0u);
                        t = fsum32(v[q].y, t);
                        t = fsum32(v[q].z, t);
                        t = fsum32(v[q].w, t);
                        pk |= (t < 31u ? t : 31u) << (8 * q);
                    }
                    uint32_t th = fsum32(hv.x, 0u);  // halo groups (lanes 0 .. 2HL-1)
                    th = fsum32(hv.y, th);
                    th = fsum32(hv.z, th);
                    th = fsum32(hv.w, th);
                    const uint32_t hl = rl_u(th, HL_ - 1), hr = rl_u(th, HL_);  // the groups beside the strip
                    uint32_t lw = dpp32<0x13C, 0xf, false>(0u, pk);  // wave_ror:1 -> lane l - 1 (lane 0: 63)
                    uint32_t rw = dpp32<0x134, 0xf, false>(0u, pk);  // wave_rol:1 -> lane l + 1 (lane 63: 0)
                    lw = lane == 0 ? (lw << 8) | (hl < 31u ? hl : 31u) : lw;
                    rw = lane == 63 ? (rw >> 8) | ((hr < 31u ? hr : 31u) << 24) : rw;
                    const uint32_t sum3 = lw + pk + rw;
                    const uint32_t k = (P.wskip + 1u) * 0x01010101u;
                    // (128 + s - k >= 128 exactly when a byte's sum s > wskip)
                    const bool over = (((sum3 | 0x80808080u) - k) & 0x80808080u) != 0u;
                    clean = __ballot(over) == 0;
                }
                if (!clean) {  // the exact chunk sums of the same registers
#pragma unroll
                    for (int q = 0; q < kLoads; ++q) {
                        const uint32_t d[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                        for (int i = 0; i < CPL; ++i) {
                            uint32_t a = 0;
#pragma unroll
                            for (int j = 0; j < DPC; ++j) a = fsum32(d[DPC * i + j], a);
                            cs[CPL * q + i] = a;
                        }
                    }
                    {
                        const uint32_t d[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
                        for (int i = 0; i < CPL; ++i) {
                            uint32_t a = 0;
#pragma unroll
                            for (int j = 0; j < DPC; ++j) a = fsum32(d[DPC * i + j], a);
                            hs[i] = a;
                        }
                    }
                    if (mesc) {  // the strip or a halo block holds an escape: where, exactly
                        uint32_t tbig = 0;
#pragma unroll
                        for (int q = 0; q < kLoads; ++q)
                            tbig = fbig_acc(v[q].w, fbig_acc(v[q].z, fbig_acc(v[q].y, fbig_acc(v[q].x, tbig))));
                        tbig = fbig_acc(hv.w, fbig_acc(hv.z, fbig_acc(hv.y, fbig_acc(hv.x, tbig))));
                        if (__ballot((tbig & kBigMask) != 0u) != 0) {
                            esc_tracks = 1;
                            any_esc = true;
                        }
                    }
                }
            }
            for (int st = 0; st < (kCheap ? 0 : NONDIR ? 2 : 1); ++st) {
                for (int k = 0; k < P.nnc; ++k) {
                    // this track's loads were issued one step ahead (pf_issue);
                    // issue the next (strip, track)'s before reducing these
                    if (!kPf) pf_issue(it, cur, st, k);
                    u32x4 v[kLoads];
#pragma unroll
                    for (int q = 0; q < kLoads; ++q) v[q] = pv[q];
                    // halos: SH chunks on each side, HL lanes per side
                    const u32x4 hv = phv;
                    pf_ok = false;
                    if (!kPf) {
                    } else if (k + 1 < P.nnc) {
                        pf_issue(it, cur, st, k + 1);
                    } else if (st + 1 < (NONDIR ? 2 : 1)) {
                        pf_issue(it, cur, st + 1, 0);
                    } else if (it + istep < it_end) {
                        uint32_t nc_ = cur;
                        while (it + istep >= units[nc_].strip0 + units[nc_].nstrips) ++nc_;
                        pf_issue(it + istep, nc_, 0, 0);
                    }
                    const uint32_t w = POOL == 2 ? cptr(P.wscreen)[k] : 1u;
                    uint32_t tbig = 0;  // this track's escape bits
#pragma unroll
                    for (int q = 0; q < kLoads; ++q) {
                        const uint32_t d[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                        for (int i = 0; i < CPL; ++i) {
                            // unweighted: the sum accumulates straight into cs
                            uint32_t a = POOL == 2 ? 0u : cs[CPL * q + i];
#pragma unroll
                            for (int j = 0; j < DPC; ++j) a = fsum32(d[DPC * i + j], a);
                            cs[CPL * q + i] = POOL == 2 ? cs[CPL * q + i] + a * w : a;
                        }
                        tbig = fbig_acc(d[3], fbig_acc(d[2], fbig_acc(d[1], fbig_acc(d[0], tbig))));
                    }
                    {
                        const uint32_t d[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
                        for (int i = 0; i < CPL; ++i) {
                            uint32_t a = POOL == 2 ? 0u : hs[i];
#pragma unroll
                            for (int j = 0; j < DPC; ++j) a = fsum32(d[DPC * i + j], a);
                            hs[i] = POOL == 2 ? hs[i] + a * w : a;
                        }
                        tbig = fbig_acc(d[3], fbig_acc(d[2], fbig_acc(d[1], fbig_acc(d[0], tbig))));
                    }
                    // wave-uniform: this track holds an escape in the strip or its halos
                    // (reading the escape tiles' index with scalar loads instead
                    // measured slower: K1a 0.34 -> 0.40 ms on configs[1])
                    const bool tesc = __ballot((tbig & kBigMask) != 0u) != 0;
                    if (tesc) {
                        const int ti = st * P.nnc + k;
                        if (ti < 64) esc_tracks |= 1ull << ti;
                        else esc_far = true;
                        any_esc = true;
                    }
                }
            }
            // Register pre-screen (no LDS): group g = lane l of load q holds
            // CPL chunks; every chunk's window of +-R chunks lies in groups
            // g-D .. g+D (D = ceil(R / CPL) <= 2), so the tag sum of those
            // groups (neighbours by wave_shr/wave_shl DPP, across loads by
            // readlane) plus both halos bounds it.  Background strips -- most
            // of the genome -- end here; the others (and any escaped field,
            // whose count the screen does not know) take the LDS screen below.
            if constexpr (kScr) {
                if (!clean && (R + CPL - 1) / CPL <= 2 && !any_esc && !pre_done) {
                    uint32_t T[kLoads];
#pragma unroll
                    for (int q = 0; q < kLoads; ++q) {
                        T[q] = 0;
#pragma unroll
                        for (int i = 0; i < CPL; ++i) T[q] += cs[CPL * q + i];
                    }
                    uint32_t hl = 0;
#pragma unroll
                    for (int i = 0; i < CPL; ++i) hl += hs[i];
                    clean = __ballot(pre_bound(T, hl) > P.wskip) == 0;
                }
            }
            if (clean) {
                mchunk = 0;
                exact_blocks = 0;
            } else {
            // A chunk holding an escaped field (a count >= kEsc stored as the
            // escape).  One pooled sample: the chunk goes exact (kBig) -- its
            // escapes sit at peaks that are exact anyway.  Several pooled
            // samples (2-bit tracks): every sample's own peaks hold escapes,
            // and sending them all exact made K1b several times longer, so the
            // chunk sum takes the chunk's true counts instead -- the escape
            // tile holds min(count, 255) of every escaped position of its
            // 1024-position block (0 elsewhere), so one 16-byte tile load per
            // chunk gives the correction (a 255 leaves the chunk unbounded,
            // kBig).  Per lane piece (64 positions, one block): the pieces'
            // tile indices are loaded together, then each piece's tile
            // chunks together -- two dependent round trips per piece, not per
            // escape.  Only strips where some lane saw an escape re-read
            // their bytes (L2).  (4-bit tracks: any count >= 8 goes exact.)
            if (any_esc) {
                constexpr bool kBound = kTB == 2 && POOL != 0;
                constexpr int NP = kLoads + 1;  // the lane's strip pieces and its halo piece
                const uint32_t nblk = ovf_nblk(U.len);
                for (int st = 0; st < (NONDIR ? 2 : 1); ++st) {
                    for (int k = 0; k < P.nnc; ++k) {
                        const int tix = st * P.nnc + k;  // only the tracks that saw an escape
                        if (tix < 64 ? !((esc_tracks >> tix) & 1ull) : !esc_far) continue;
                        const uint32_t trk = (uint32_t)(st * S + ncs[k]);
                        const uint32_t w = POOL == 2 ? cptr(P.wscreen)[k] : 1u;
                        gu32x4 *t = (gu32x4 *)(track_u8(U, S, st, ncs[k]) + fbyte(kPadPos + p0 - 1));
                        const bool hl_ok = lane < 2 * HL;
                        const int hl = lane < HL ? lane - HL : kLoads * kWave + lane - HL;
                        u32x4 x[NP];
#pragma unroll
                        for (int q = 0; q < kLoads; ++q) x[q] = t[64 * q + lane];
                        x[kLoads] = hl_ok ? t[hl] : u32x4{0u, 0u, 0u, 0u};
                        uint32_t em[NP];  // chunks of each piece holding an escape
#pragma unroll
                        for (int q = 0; q < NP; ++q) {
                            const uint32_t d[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
                            em[q] = 0;
#pragma unroll
                            for (int i = 0; i < CPL; ++i) {
                                uint32_t e = 0;
#pragma unroll
                                for (int j = 0; j < DPC; ++j) e |= fbig32(d[DPC * i + j]);
                                em[q] |= (e ? 1u : 0u) << i;
                            }
                        }
                        if constexpr (!kBound) {
#pragma unroll
                            for (int q = 0; q < kLoads; ++q) big |= em[q] << (CPL * q);
                            hbig |= em[kLoads];
                        } else {
                            // first position of each piece (16 bytes = 64 positions)
                            auto ppos = [&](int q) -> int64_t {
                                return p0 + (int64_t)kPerByte * 16 * (q < kLoads ? 64 * q + lane : hl);
                            };
                            uint32_t ti[NP];
#pragma unroll
                            for (int q = 0; q < NP; ++q) {
                                ti[q] = kNoTile;
                                const int64_t pp = ppos(q);
                                if (em[q] && U.ovf_tidx && pp >= 1 && pp <= (int64_t)U.len)
                                    ti[q] = ((const uint32_t *)U.ovf_tidx)[(size_t)trk * nblk +
                                                                           ((uint32_t)(pp - 1) >> kOvfBlkShift)];
                            }
#pragma unroll
                            for (int q = 0; q < NP; ++q) {
                                if (!em[q]) continue;
                                if (ti[q] == kNoTile) {  // cannot happen for a stored escape: stay exact
                                    if (q < kLoads) big |= em[q] << (CPL * q);
                                    else hbig |= em[q];
                                    continue;
                                }
                                const uint8_t *tile = (const uint8_t *)U.ovf_tiles + (size_t)ti[q] * kOvfBlk +
                                                      ((uint32_t)(ppos(q) - 1) & (kOvfBlk - 1u));
                                u32x4 tv[CPL];
#pragma unroll
                                for (int i = 0; i < CPL; ++i)
                                    if ((em[q] >> i) & 1u) tv[i] = *(const u32x4 *)(tile + 16 * i);
                                const uint32_t d[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
                                for (int i = 0; i < CPL; ++i) {
                                    if (!((em[q] >> i) & 1u)) continue;
                                    const uint32_t v[4] = {tv[i].x, tv[i].y, tv[i].z, tv[i].w};
                                    uint32_t tsum = 0, full = 0;
#pragma unroll
                                    for (int m = 0; m < 4; ++m) {
                                        tsum = __builtin_amdgcn_sad_u8(v[m], 0u, tsum);
                                        const uint32_t nv = ~v[m];  // a byte of 255 (count >= 255)
                                        full |= (nv - 0x01010101u) & ~nv & 0x80808080u;
                                    }
                                    uint32_t nesc = 0;
#pragma unroll
                                    for (int j = 0; j < DPC; ++j) nesc += (uint32_t)__builtin_popcount(fbig32(d[DPC * i + j]));
                                    const uint32_t corr = (tsum - kEsc * nesc) * w;
                                    if (q < kLoads) {
                                        if (full) big |= 1u << (CPL * q + i);
                                        else cs[CPL * q + i] += corr;
                                    } else {
                                        if (full) hbig |= 1u << i;
                                        else hs[i] += corr;
                                    }
                                }
                            }
                        }
                    }
                }
            }
            // (a lane's CPL chunks never straddle a pad word: CPL divides 16)
#pragma unroll
            for (int q = 0; q < kLoads; ++q) {
                uint32_t *d = scr + scr_at(kScrHalo + kWave * CPL * q + CPL * lane);
#pragma unroll
                for (int i = 0; i < CPL; ++i) d[i] = ((big >> (CPL * q + i)) & 1u) ? kBig : cs[CPL * q + i];
            }
            if (lane < 2 * HL) {
                uint32_t *d = scr + scr_at(lane < HL ? kScrHalo - SH + CPL * lane
                                                     : kScrHalo + kBlocks * kWave + CPL * (lane - HL));
#pragma unroll
                for (int i = 0; i < CPL; ++i) d[i] = ((hbig >> i) & 1u) ? kBig : hs[i];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t *rd = scr + 17 * lane;  // index 16l + j = word 17l + j + j/16
            const uint32_t m = screen_any<4 * NH>(R, rd, P.wskip, P.fw, P.fthr);
            const uint64_t lanes = __ballot(m != 0u);  // lane l covers chunks 16l..16l+15
            mchunk = m;
            exact_blocks = 0;
#pragma unroll
            for (int bk = 0; bk < kBlocks; ++bk)
                exact_blocks |= ((lanes >> (4 * bk)) & 0xFull) ? (1u << bk) : 0u;
            // the next strip reuses scr only after every lane has read it
            __builtin_amdgcn_wave_barrier();
            }  // !clean
        }
        if constexpr (kScr) {
            if (exact_blocks == 0) {  // no run can touch this strip
                const uint64_t info = ((uint64_t)(local == 0) << 34) | ((uint64_t)(local + 1 == unstrips) << 35);
                if (lane == 0) P.strip_info[strip] = info;
            } else {
                // into this wave's stash: multi-block strips from its front,
                // single-block ones from its back (xref_kernel lists them)
                const bool front = __builtin_popcount(exact_blocks) >= kXFront;
                const uint32_t slot = wave * P.xcap + (front ? xnf++ : P.xcap - 1u - xnb++);
                uint32_t *e = P.xlist + (uint64_t)slot * kXEntry;
                const uint32_t hi = (uint32_t)__shfl_down((int)mchunk, 1);
                if ((lane & 1) == 0) e[2 + (lane >> 1)] = mchunk | (hi << 16);
                if (lane == 0) { e[0] = strip; e[1] = exact_blocks | ((cur < 0xFFFFu ? cur : 0xFFFFu) << 16); }
            }
            continue;
        }

        // Run state of the strip, wave-uniform (scalar registers): the flag
        // loop below visits only live words, so a run that reaches the end of
        // the last visited word and finds no flag in the next visited one
        // ended at that word's last position.
        RecList R_{0, 0, kInline};
        uint64_t F0 = 0;
        bool open = false;      // a run is open at the last position of word `last`
        int last = -2;          // strip word index (0..255) of the last visited live word
        bool pk_ok = false;     // the open run started inside this strip
        // the open run's first largest key, its position, and whether a
        // second position holds the same key (Q keys: K3 then orders the tied
        // positions by their FP64 scores; marked by +0.5)
        double best = -__builtin_inf();
        uint32_t bpos = 0;
        bool btie = false;
        auto run_key = [&]() { return (kQ && qm && btie) ? best + 0.5 : best; };
        auto close_run = [&](uint32_t end_pos) {
            const double m = run_key();
            rec_end(R_, end_pos, pk_ok ? bpos : 0u, m, P, strip, lane);
            if (!pk_ok && lane == 0) {  // the run open at p0: its part in this strip
                P.spk[4ull * strip] = (uint64_t)__double_as_longlong(m);
                P.spk[4ull * strip + 1] = bpos;
            }
            open = false;
        };

        for (uint32_t eb = exact_blocks; eb; eb &= eb - 1u) {
            const int j = __builtin_ctz(eb);  // blocks without a flag are never visited
            // words of this block that can hold a flag (the others keep F = 0
            // and receive no scatter)
            uint32_t lw = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // word w = 4i + q of the block <- lane 4j + i, nibble q
                const uint64_t bq = __ballot(((mchunk >> (4 * q)) & 0xFu) != 0u) >> (4 * j);
#pragma unroll
                for (int i = 0; i < 4; ++i) lw |= (uint32_t)((bq >> i) & 1ull) << (4 * i + q);
            }
#ifdef UPK_DEBUG_COUNTS
            if (lane == 0) {
                atomicAdd(&P.dbg[0], 1ull);
                atomicAdd(&P.dbg[1], (unsigned long long)__builtin_popcount(lw));
            }
#endif
            const int64_t x0 = p0 + 64 * (j * SW - NH);  // position of window word 0, lane 0
#if defined(UPK_DEBUG_COUNTS) || defined(UPK_DEBUG_TIMES)
            const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
            T wf[NWIN], wr[NONDIR ? NWIN : 1];
            load_words_staged<NWIN, POOL>(wf, U, S, 0, x0, lane, P.nnc, P.nc, P.coef, (uint8_t *)scs);
            if constexpr (NONDIR)
                load_words_staged<NWIN, POOL>(wr, U, S, 1, x0, lane, P.nnc, P.nc, P.coef,
                                              (uint8_t *)scs + kStageBytes);
            // the hit bitmaps of the window words are ballots taken where they
            // are used (Q scans, FP64 walk), not held for the whole block: 2 x
            // NWIN SGPRs live across the block made the compiler spill SGPRs
            // into VGPR lanes (K1b 65 -> 79 M VALU per launch when NWIN's
            // kernels widened to NH <= 8)
#ifdef UPK_DEBUG_TIMES
            const uint64_t tq1 = __builtin_amdgcn_s_memtime();
            dt_load += tq1 - tq0;
#endif
#ifdef UPK_DEBUG_COUNTS
            const uint64_t tq1 = __builtin_amdgcn_s_memtime();
            if (lane == 0) {
                uint32_t nh = 0;
                for (int w = 0; w < NWIN; ++w) nh += __builtin_popcountll(__ballot(nz(wf[w])));
                atomicAdd(&P.dbg[2], (unsigned long long)nh);
                atomicAdd(&P.dbg[3], (unsigned long long)(tq1 - tq0));
            }
#endif
            // ---- K1b keys: exact integer Q of every live word ----
            // Q(x) = sum over hits h within bw of c_h (bw^2 - (x-h)^2), from
            // wave prefix sums of c, c*j, c*j^2 over the window (j = window
            // index; uint32 wrap arithmetic is exact since Q < 2^32, which
            // the host guarantees).  score(x) = alpha * Q(x) * (1 +- delta)
            // for the FP64 weights and any summation order, so Q <= qno
            // proves no flag, Q >= qyes a flag, and distinct Q order the
            // FP64 scores (delta * Q << 1): only words with an undecided
            // lane go through the FP64 walk below.
            uint32_t xw = lw;          // output words the FP64 walk computes
            uint32_t qv[kQ ? SW : 1];  // Q at each live word's lane position
            if constexpr (kQ) {
                if (qm) {
                    xw = 0;
                    uint32_t P0[NWIN], P1[NWIN], P2[NWIN];
                    // the prefix sums start at the first live word's window
                    // (W is a difference of two prefixes: any common base
                    // cancels) and end with the last one's
                    uint32_t c0 = 0, c1 = 0, c2 = 0;  // totals of the words before
                    // window words some live word reads (output word k reads
                    // window words k .. k + 2NH); no window spans a word
                    // outside them, so the base restarts there
                    uint32_t nd = lw;
#pragma unroll
                    for (int d = 1; d <= 2 * NH; ++d) nd |= lw << d;
                    WordLoop<0, NWIN>::run([&](auto wc) {
                        constexpr int w = decltype(wc)::value;
                        uint64_t any = 0;
                        if ((nd >> w) & 1u) {
                            if constexpr (NONDIR) any = __ballot(nz(wf[w]) || nz(wr[NONDIR ? w : 0]));
                            else any = __ballot(nz(wf[w]));
                        } else {
                            c0 = c1 = c2 = 0u;
                        }
                        if (any == 0) {
                            P0[w] = c0;
                            P1[w] = c1;
                            P2[w] = c2;
                        } else {
                            uint32_t c = (uint32_t)wf[w];
                            if constexpr (NONDIR) c += (uint32_t)wr[NONDIR ? w : 0];
                            const uint32_t j = 64u * w + (uint32_t)lane;
                            const uint32_t s0 = wave_scan_u32(c), s1 = wave_scan_u32(c * j),
                                           s2 = wave_scan_u32(c * (j * j));
                            P0[w] = s0 + c0;
                            P1[w] = s1 + c1;
                            P2[w] = s2 + c2;
                            c0 += rl_u(s0, 63);
                            c1 += rl_u(s1, 63);
                            c2 += rl_u(s2, 63);
                        }
                        constexpr int k = w - 2 * NH;  // output word whose window ends with word w
                        if constexpr (k >= 0) {
                            if ((lw >> k) & 1u) {
                                auto win = [&](const uint32_t (&Pa)[NWIN]) {
                                    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(
                                        hadr, (int)(hsel ? Pa[k + 2 * NH] : Pa[k + 2 * NH - 1]));
                                    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(
                                        ladr, (int)(lsel ? Pa[k + 1] : Pa[k]));
                                    return hi - lo;
                                };
                                const uint32_t W0 = win(P0), W1 = win(P1), W2 = win(P2);
                                const uint32_t i = 64u * (k + NH) + (uint32_t)lane;
                                const uint32_t q = bw2 * W0 - (i * i) * W0 + 2u * i * W1 - W2;
                                qv[k] = q;
                                if (__ballot(q > P.qno && q < P.qyes)) xw |= 1u << k;
                            } else {
                                qv[k] = 0;
                            }
                        }
                    });
                }
            }
#ifdef UPK_DEBUG_TIMES
            dt_q += __builtin_amdgcn_s_memtime() - tq1;
#endif
            // ---- KDE: scatter every hit of the window, ascending ----
            double af[SW], ar[NONDIR ? SW : 1];
#pragma unroll
            for (int k = 0; k < SW; ++k) {
                af[k] = 0.0;
                if constexpr (NONDIR) ar[k] = 0.0;
            }
            WordLoop<0, NWIN>::run([&](auto wc) {
                constexpr int W = decltype(wc)::value;
                // output words a hit of window word W reaches: W-2NH .. W
                constexpr int OLO = W - 2 * NH < 0 ? 0 : W - 2 * NH;
                constexpr int OHI = W > SW - 1 ? SW - 1 : W;
                const uint32_t reach = xw & (((2u << OHI) - 1u) & ~((1u << OLO) - 1u));
                if (!reach) return;
                uint64_t m = __ballot(nz(wf[W]));
                if constexpr (W < NH) m &= edge_lo[W];
                if constexpr (W >= NH + SW) m &= edge_hi[W - NH - SW];
                while (m) {
                    int hb[kHB];
                    double hc[kHB];
                    next_hits(m, wf[W], hb, hc);
                    scatter_hits<NH, SW, W>(af, hb, hc, lane, bw, ktab, reach);
                }
                if constexpr (NONDIR) {
                    uint64_t q = __ballot(nz(wr[W]));
                    if constexpr (W < NH) q &= edge_lo[W];
                    if constexpr (W >= NH + SW) q &= edge_hi[W - NH - SW];
                    while (q) {
                        int hb[kHB];
                        double hc[kHB];
                        next_hits(q, wr[W], hb, hc);
                        scatter_hits<NH, SW, W>(ar, hb, hc, lane, bw, ktab, reach);
                    }
                }
            });
#ifdef UPK_DEBUG_COUNTS
            const uint64_t tq2 = __builtin_amdgcn_s_memtime();
            if (lane == 0) atomicAdd(&P.dbg[4], (unsigned long long)(tq2 - tq1));
#endif
#ifdef UPK_DEBUG_TIMES
            const uint64_t tq2 = __builtin_amdgcn_s_memtime();
            dt_scat += tq2 - tq1;
#endif
            double sc[SW];
            double mx = -__builtin_inf();
#pragma unroll
            for (int k = 0; k < SW; ++k) {
                // a dead word holds no flag (the screen's proof): no key, no
                // LDS store (the flag loop skips it) -- 3/4 of a block's words
                if constexpr (!PROF) {
                    if (!((lw >> k) & 1u)) {
                        sc[k] = -1.0;
                        continue;
                    }
                }
                if constexpr (NONDIR) sc[k] = af[k] + ar[k];  // forwardScore + reverseScore
                else sc[k] = af[k];
                if constexpr (!PROF) {
                    if (kQ && qm) {
                        // key = Q of a flagged position (proven by Q, or by the
                        // FP64 score of an undecided lane), -1 otherwise
                        const uint32_t q = qv[kQ ? k : 0];
                        const bool fl = q >= P.qyes || (q > P.qno && sc[k] >= P.thr);
                        sc[k] = (((lw >> k) & 1u) && fl) ? (double)q : -1.0;
                    } else {
                        sc[k] = ((lw >> k) & 1u) ? sc[k] : -1.0;  // dead word: no flag
                    }
                }
                mx = __builtin_fmax(mx, sc[k]);
            }
            if constexpr (PROF) {
#pragma unroll
                for (int k = 0; k < SW; ++k) {
                    const int64_t q = p0 + 64 * (j * SW + k) + lane - P.prof_first;
                    if (q >= 0 && q < (int64_t)P.prof_len) {
                        P.prof_f[q] = af[k];
                        if constexpr (NONDIR) P.prof_r[q] = ar[k];
                    }
                }
            } else {
                // ---- flags and run boundaries (only blocks touching a run) ----
#ifdef UPK_DEBUG_COUNTS
                {
                    uint32_t fw = 0, fp = 0, hw = 0;
                    for (int k = 0; k < SW; ++k) {
                        const uint64_t Fk = __ballot(sc[k] >= P.thr);
                        fw += Fk != 0;
                        fp += __builtin_popcountll(Fk);
                        hw += __ballot(sc[k] >= 0.5 * P.thr) != 0;
                    }
                    if (lane == 0) {
                        atomicAdd(&P.dbg[5], (unsigned long long)fw);
                        atomicAdd(&P.dbg[6], (unsigned long long)fp);
                        atomicAdd(&P.dbg[7], (unsigned long long)hw);
                    }
                }
#endif
                const uint64_t anyflag = __ballot(mx >= kthr);
                if (anyflag || open) {
                    // keys / scores through LDS so the word loop below stays a
                    // loop (unrolled, its run bookkeeping overflows the I-cache)
#pragma unroll
                    for (int k = 0; k < SW; ++k) {
                        if (!((lw >> k) & 1u)) continue;  // never read (dead word)
                        scs[64 * k + lane] = sc[k];
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
                    for (uint32_t lm = lw; lm; lm &= lm - 1u) {
                        const int k = __builtin_ctz(lm);
                        const int g = j * SW + k;  // word of the strip
                        const int64_t wpos = p0 + 64 * g;
                        // a run open at the end of an earlier word met a word
                        // without flags before this one: it ended there
                        if (open && g != last + 1) close_run((uint32_t)(p0 + 64 * (last + 1) - 1));
                        last = g;
                        const double sck = scs[64 * k + lane];
                        const uint64_t F = __ballot(sck >= kthr);
                        if (g == 0) F0 = F;
                        if (open && !(F & 1ull)) close_run((uint32_t)(wpos - 1));
                        // no interior start at p0 (K2 joins it to the previous strip's run)
                        uint64_t st = F & ~((F << 1) | ((open || g == 0) ? 1ull : 0ull));
                        while (st) {
                            const int b = __builtin_ctzll(st);
                            st &= st - 1;
                            rec_start(R_, (uint32_t)(wpos + b), P, strip, lane);
                        }
                        // each maximal segment of F: its largest key and the
                        // lanes holding it (Region::addPos keeps the first
                        // maximum, data.cpp:98-101), merged into the run's
                        uint64_t rem = F;
                        while (rem) {
                            const int a = __builtin_ctzll(rem);
                            const uint64_t up = ~(rem >> a);
                            const int len = up ? __builtin_ctzll(up) : 64 - a;
                            rem = len + a >= 64 ? 0ull : rem & (~0ull << (a + len));
                            const bool in = lane >= a && lane < a + len;
                            double m;
                            uint64_t at;
                            if (kQ && qm) {  // integer keys >= 1
                                const uint32_t kq = in ? (uint32_t)sck : 0u;
                                const uint32_t mq = wave_max_u32(kq);
                                at = __ballot(kq == mq);
                                m = (double)mq;
                            } else {
                                m = wave_max_d(in ? sck : -__builtin_inf());
                                at = __ballot(in && sck == m);
                            }
                            if (!(a == 0 && open)) {  // a new run
                                best = m;
                                bpos = (uint32_t)(wpos + __builtin_ctzll(at));
                                btie = (at & (at - 1)) != 0;
                                pk_ok = g != 0 || a != 0;  // one at p0 may continue the previous strip
                            } else if (m > best) {
                                best = m;
                                bpos = (uint32_t)(wpos + __builtin_ctzll(at));
                                btie = (at & (at - 1)) != 0;
                            } else if (m == best) {
                                btie = true;
                            }
                            open = true;
                            if (a + len < 64) close_run((uint32_t)(wpos + a + len - 1));
                        }
                    }
                    __builtin_amdgcn_wave_barrier();  // scs reused by the next block
                }
            }
#ifdef UPK_DEBUG_TIMES
            dt_flag += __builtin_amdgcn_s_memtime() - tq2;
#endif
        }
        if constexpr (PROF) continue;
        // a run open at the end of the last visited word: it ends there,
        // unless that word is the strip's last (K2 joins it to the next strip)
        if (open && last != kStripWords - 1) close_run((uint32_t)(p0 + 64 * (last + 1) - 1));
        if (open) {  // the run open at the strip's last position: its part here
            if (lane == 0) {
                P.spk[4ull * strip + 2] = (uint64_t)__double_as_longlong(run_key());
                P.spk[4ull * strip + 3] = bpos;
            }
        }
        const uint64_t info = (uint64_t)R_.ns | ((uint64_t)R_.ne << 16) | ((F0 & 1ull) << 32) |
                              ((uint64_t)open << 33) | ((uint64_t)(local == 0) << 34) |
                              ((uint64_t)(local + 1 == unstrips) << 35) |
                              ((uint64_t)(R_.slot != kInline) << 36);
        if (lane == 0) P.strip_info[strip] = info;
#ifdef UPK_DEBUG_TIMES
        dt_item += __builtin_amdgcn_s_memtime() - t_it0;
#endif
    }
#ifdef UPK_DEBUG_TIMES
    if (MODE == kModeExact && lane == 0 && P.dbg) {
        atomicAdd(&P.dbg[16], (unsigned long long)dt_item);
        atomicAdd(&P.dbg[17], (unsigned long long)dt_load);
        atomicAdd(&P.dbg[18], (unsigned long long)dt_scat);
        atomicAdd(&P.dbg[19], (unsigned long long)dt_flag);
        atomicAdd(&P.dbg[20], (unsigned long long)n_items);
        atomicMax(&P.dbg[21], (unsigned long long)dt_item);
        atomicAdd(&P.dbg[22], 1ull);
        atomicAdd(&P.dbg[23], (unsigned long long)dt_q);
    }
#endif
    if constexpr (kScr) {
        if (lane == 0) {
            P.xwcount[2 * wave] = xnf;
            P.xwcount[2 * wave + 1] = xnb;
        }
    }
}

// ------------------------------------------------------------------------
// K1a over the 2-bit fields of ONE pooled directional track (POOL 0), the
// pass without the per-dataset index (kModeScreenF, DESIGN.md §3 "Index
// policy") -- configs[1]'s cold pass.  Same outputs as scan_kernel's screen
// (strip summaries of clean strips, work-list stash entries of the others),
// built for the stream:
//  * each wave screens a contiguous run of strips; a cursor walks the unit
//    table (one scalar load per unit, not per strip), so no load address
//    waits on a scalar load;
//  * three strip buffers in rotation (the loop is unrolled by three, each
//    buffer a fixed set of registers): the loads of strips i+1 and i+2 are
//    in flight while strip i is screened -- scan_kernel's kCheap path copied
//    its prefetch buffer each strip, which waited for every load of the wave
//    (vmcnt(0)) and then for the next strip's unit-table loads before
//    issuing the next loads: one strip in flight per wave, SQ_WAIT_ANY 60 %
//    of the wave cycles (profiles/r06/);
//  * the packed pre-screen (scan_kernel's, R <= 4) settles background
//    strips; the others take chunk sums, escape bits and the LDS screen.
#ifndef UPK_K1AF_DEPTH
#define UPK_K1AF_DEPTH 3  // strip buffers in rotation (2 or 3)
#endif
template <int NH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UPK_K1A_WPE)))
k1a_fields_kernel(ScanParams P, uint32_t strip_begin, uint32_t strip_end) {
    extern __shared__ double lds_[];
    uint32_t *scr = (uint32_t *)lds_ + (threadIdx.x >> 6) * kScrWords;
    constexpr int CPL = 16 / kChunkBytes;           // chunks per 16-byte lane load (4)
    constexpr int kLoads = kStripBytes / (kWave * 16);
    constexpr int SH = scr_halo(NH);                // screen halo chunks per side (16)
    constexpr int HL = SH * kChunkBytes / 16;       // halo lane loads per side (4)
    static_assert(kTB == 2 && CPL == 4 && kChunkBytes == 4 && kLoads == 4, "2-bit layout");
    const auto *units = cptr(P.units);
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const int R = (P.bw + kChunk - 1) / kChunk;
    const int S = P.S;
    const int nc0 = cptr(P.nc)[0];
    const uint32_t wskip = P.wskip;
    const bool packed_ok = R <= CPL && wskip < 31u;
    const uint32_t nsr = strip_end - strip_begin;
    const uint32_t per = (nsr + nwaves - 1) / nwaves;
    const uint32_t off = (uint64_t)wave * per < nsr ? wave * per : nsr;
    const uint32_t it0 = strip_begin + off;
    const uint32_t it_end = it0 + per < strip_end ? it0 + per : strip_end;
    const auto *eb = cptr(P.esc);  // (constant address space: scalar loads)
    const uint32_t esc_row = (uint32_t)nc0 * P.esc_nw;  // strand 0, the pooled sample
    uint32_t xnf = 0, xnb = 0;

    struct Buf {
        u32x4 v[4];
        u32x4 h;
    };
    // prefetch cursor (the unit of the strip being issued)
    uint32_t pc_u = 0, pc_s0 = 0, pc_end = 0;
    gu8 *pc_base = nullptr;
    auto issue = [&](uint32_t strip, Buf &b) {
        while (strip >= pc_end) {
            pc_u = pc_end == 0 ? find_unit(units, P.nunits, strip) : pc_u + 1;
            const UnitDesc Un = units[pc_u];
            pc_s0 = Un.strip0;
            pc_end = Un.strip0 + Un.nstrips;
            pc_base = track_u8(Un, S, 0, nc0) + fbyte(kPadPos);  // position 1
        }
        gu32x4 *t = (gu32x4 *)(pc_base + (uint64_t)(strip - pc_s0) * kStripBytes);
#pragma unroll
        for (int q = 0; q < 4; ++q) b.v[q] = __builtin_nontemporal_load(t + 64 * q + lane);
        // (every lane loads -- lanes past the halo repeat the right halo's
        // pieces and drop them -- so no load is under a branch and the
        // compiler can count the loads still in flight exactly)
        const u32x4 h = t[lane < HL ? lane - HL : kLoads * kWave + ((lane - HL) & (HL - 1))];
        b.h = lane < 2 * HL ? h : u32x4{0u, 0u, 0u, 0u};
    };
    // current cursor (the unit of the strip being screened)
    uint32_t c_u = 0, c_s0 = 0, c_end = 0;

    auto screen = [&](uint32_t strip, const Buf &b) {
        while (strip >= c_end) {
            c_u = c_end == 0 ? find_unit(units, P.nunits, strip) : c_u + 1;
            c_s0 = units[c_u].strip0;
            c_end = c_s0 + units[c_u].nstrips;
        }
        const uint32_t local = strip - c_s0, unstrips = c_end - c_s0;
        // the strip's escape bit (a scalar load: its wait never holds the
        // vector loads in flight; 32 strips share a word)
        const uint32_t escw = eb ? eb[esc_row + (strip >> 5)] : ~0u;
        const bool mesc = (escw >> (strip & 31u)) & 1u;
        bool clean = false, pre_done = false;
        if (packed_ok && !mesc) {  // (scan_kernel's packed pre-screen; see there)
            pre_done = true;
            uint32_t pk = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t t = fsum32(b.v[q].x, 0u);
                t = fsum32(b.v[q].y, t);
                t = fsum32(b.v[q].z, t);
                t = fsum32(b.v[q].w, t);
                pk |= (t < 31u ? t : 31u) << (8 * q);
            }
            uint32_t th = fsum32(b.h.x, 0u);
            th = fsum32(b.h.y, th);
            th = fsum32(b.h.z, th);
            th = fsum32(b.h.w, th);
            const uint32_t hl = rl_u(th, HL - 1), hr = rl_u(th, HL);
            uint32_t lw = dpp32<0x13C, 0xf, false>(0u, pk);  // wave_ror:1
            uint32_t rw = dpp32<0x134, 0xf, false>(0u, pk);  // wave_rol:1
            lw = lane == 0 ? (lw << 8) | (hl < 31u ? hl : 31u) : lw;
            rw = lane == 63 ? (rw >> 8) | ((hr < 31u ? hr : 31u) << 24) : rw;
            const uint32_t sum3 = lw + pk + rw;
            const uint32_t k = (wskip + 1u) * 0x01010101u;
            clean = __ballot((((sum3 | 0x80808080u) - k) & 0x80808080u) != 0u) == 0;
        }
        uint32_t mchunk = 0, exact_blocks = 0;
        if (!clean) {
            uint32_t cs[16], hs[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t d[4] = {b.v[q].x, b.v[q].y, b.v[q].z, b.v[q].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) cs[4 * q + i] = fsum32(d[i], 0u);
            }
            {
                const uint32_t d[4] = {b.h.x, b.h.y, b.h.z, b.h.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) hs[i] = fsum32(d[i], 0u);
            }
            // a chunk holding an escaped field goes exact (one pooled
            // sample: its escapes sit at peaks that are exact anyway)
            uint32_t big = 0, hbig = 0;
            if (mesc) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t d[4] = {b.v[q].x, b.v[q].y, b.v[q].z, b.v[q].w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) big |= (fbig32(d[i]) ? 1u : 0u) << (4 * q + i);
                }
                const uint32_t d[4] = {b.h.x, b.h.y, b.h.z, b.h.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) hbig |= (fbig32(d[i]) ? 1u : 0u) << i;
            }
            // scan_kernel's register pre-screen over groups g-D .. g+D (D = 2)
            if (!pre_done && !mesc && (R + CPL - 1) / CPL <= 2) {
                uint32_t T[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) T[q] = cs[4 * q] + cs[4 * q + 1] + cs[4 * q + 2] + cs[4 * q + 3];
                const uint32_t hsum = hs[0] + hs[1] + hs[2] + hs[3];
                uint32_t htot = 0;
#pragma unroll
                for (int l = 0; l < 2 * HL; ++l) htot += rl_u(hsum, l);
                const int D = (R + CPL - 1) / CPL;
                uint32_t bmax = 0;
                uint32_t l1[4], r1[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    l1[q] = dpp32<0x138, 0xf, false>(0u, T[q]);
                    r1[q] = dpp32<0x130, 0xf, false>(0u, T[q]);
                    const uint32_t lf = q > 0 ? rl_u(T[q > 0 ? q - 1 : 0], 63) : 0u;
                    const uint32_t rf = q + 1 < 4 ? rl_u(T[q + 1 < 4 ? q + 1 : q], 0) : 0u;
                    l1[q] = lane == 0 ? lf : l1[q];
                    r1[q] = lane == 63 ? rf : r1[q];
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t bq = T[q] + l1[q] + r1[q];
                    if (D == 2) {
                        uint32_t l2 = dpp32<0x138, 0xf, false>(0u, l1[q]);
                        uint32_t r2 = dpp32<0x130, 0xf, false>(0u, r1[q]);
                        const uint32_t lf = q > 0 ? rl_u(l1[q > 0 ? q - 1 : 0], 63) : 0u;
                        const uint32_t rf = q + 1 < 4 ? rl_u(r1[q + 1 < 4 ? q + 1 : q], 0) : 0u;
                        l2 = lane == 0 ? lf : l2;
                        r2 = lane == 63 ? rf : r2;
                        bq += l2 + r2;
                    }
                    bmax = bq > bmax ? bq : bmax;
                }
                clean = __ballot(bmax + htot > wskip) == 0;
            }
            if (!clean) {  // the LDS screen (scan_kernel's layout and screen_any)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t *d = scr + scr_at(kScrHalo + kWave * CPL * q + CPL * lane);
#pragma unroll
                    for (int i = 0; i < 4; ++i) d[i] = ((big >> (4 * q + i)) & 1u) ? kBig : cs[4 * q + i];
                }
                if (lane < 2 * HL) {
                    uint32_t *d = scr + scr_at(lane < HL ? kScrHalo - SH + CPL * lane
                                                         : kScrHalo + kBlocks * kWave + CPL * (lane - HL));
#pragma unroll
                    for (int i = 0; i < 4; ++i) d[i] = ((hbig >> i) & 1u) ? kBig : hs[i];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t *rd = scr + 17 * lane;  // index 16l + j = word 17l + j + j/16
                const uint32_t m = screen_any<4 * NH>(R, rd, wskip, P.fw, P.fthr);
                const uint64_t lanes = __ballot(m != 0u);
                mchunk = m;
#pragma unroll
                for (int bk = 0; bk < kBlocks; ++bk)
                    exact_blocks |= ((lanes >> (4 * bk)) & 0xFull) ? (1u << bk) : 0u;
                __builtin_amdgcn_wave_barrier();  // the next strip reuses scr after every lane read it
            }
        }
        if (exact_blocks == 0) {  // no run can touch this strip
            const uint64_t info = ((uint64_t)(local == 0) << 34) | ((uint64_t)(local + 1 == unstrips) << 35);
            if (lane == 0) P.strip_info[strip] = info;
        } else {
            const bool front = __builtin_popcount(exact_blocks) >= kXFront;
            const uint32_t slot = wave * P.xcap + (front ? xnf++ : P.xcap - 1u - xnb++);
            uint32_t *e = P.xlist + (uint64_t)slot * kXEntry;
            const uint32_t hi = (uint32_t)__shfl_down((int)mchunk, 1);
            if ((lane & 1) == 0) e[2 + (lane >> 1)] = mchunk | (hi << 16);
            if (lane == 0) { e[0] = strip; e[1] = exact_blocks | ((c_u < 0xFFFFu ? c_u : 0xFFFFu) << 16); }
        }
    };

    // (loads past the run repeat its last strip: unconditional issues keep
    // the in-flight count exact, so each screen waits for its own buffer only)
    // (UPK_K1AF_DEPTH 2: one strip in flight beside the screened one)
    if (it0 < it_end) {
        const uint32_t last = it_end - 1;
        auto cl = [&](uint32_t x) { return x < last ? x : last; };
#if UPK_K1AF_DEPTH == 2
        Buf b0, b1;
        issue(it0, b0);
        for (uint32_t it = it0;; it += 2) {
            issue(cl(it + 1), b1);
            screen(it, b0);
            if (it + 1 > last) break;
            issue(cl(it + 2), b0);
            screen(it + 1, b1);
            if (it + 2 > last) break;
        }
#else
        Buf b0, b1, b2;
        issue(it0, b0);
        issue(cl(it0 + 1), b1);
        for (uint32_t it = it0;; it += 3) {
            issue(cl(it + 2), b2);
            screen(it, b0);
            if (it + 1 > last) break;
            issue(cl(it + 3), b0);
            screen(it + 1, b1);
            if (it + 2 > last) break;
            issue(cl(it + 4), b1);
            screen(it + 2, b2);
            if (it + 3 > last) break;
        }
#endif
    }
    if (lane == 0) {
        P.xwcount[2 * wave] = xnf;
        P.xwcount[2 * wave + 1] = xnb;
    }
}

#ifndef UPK_NH_TU  // the per-NH translation units hold only the templated kernels
// ------------------------------------------------------------------------
// K1q: the region scan of a threshold <= 0 (quirk Q11 live), parallel.
// With thr <= 0 and non-negative scores every processed position qualifies,
// so processPosition (misc/peakcall.cpp:55-86) turns every maximal run of
// processed positions -- the positions within bw of an add() (any sample,
// controls included: control-only adds retire positions too; both strands
// of a nondirectional unit) -- into one region, reached by a leap: the
// run's first position joins without setting `left` (peakcall.cpp:76-78),
// so the host shifts the run's coordinates by one.  This
// kernel writes each strip's run boundaries in K1b's record format (peaks
// unknown: K3 runs its KDE), so K2 and K3 follow unchanged.  A run starts at
// a - bw for an add a with no add in [a - 2bw - 1, a - 1] and ends at a + bw
// for an add with none in [a + 1, a + 2bw + 1].  One wave per strip: 64-
// position presence words of the strip and a kQHalo-word halo on each side
// (bw <= kMaxBw), five words per lane; the previous / next add of every word
// by wave scans.  2-bit tracks (the host checks).
__device__ __forceinline__ uint64_t nz_bits64(u32x4 x) {
    auto c16 = [](uint32_t d) {  // nonzero 2-bit fields -> 16 bits
        uint32_t v = (d | (d >> 1)) & 0x55555555u;
        v = (v | (v >> 1)) & 0x33333333u;
        v = (v | (v >> 2)) & 0x0F0F0F0Fu;
        v = (v | (v >> 4)) & 0x00FF00FFu;
        v = (v | (v >> 8)) & 0x0000FFFFu;
        return (uint64_t)v;
    };
    return c16(x.x) | (c16(x.y) << 16) | (c16(x.z) << 32) | (c16(x.w) << 48);
}

__device__ __forceinline__ uint64_t rl_u64(uint64_t v, int l) {
    return (uint64_t)rl_u((uint32_t)v, l) | ((uint64_t)rl_u((uint32_t)(v >> 32), l) << 32);
}

// bits of word [base, base + 63] inside [lo, hi]
__device__ __forceinline__ uint64_t range_bits(int64_t base, int64_t lo, int64_t hi) {
    const int64_t a = lo > base ? lo - base : 0, b = hi < base + 63 ? hi - base : 63;
    if (a > b) return 0;
    const uint64_t up = b == 63 ? ~0ull : ((1ull << (b + 1)) - 1);
    return up & ~((1ull << a) - 1);
}

constexpr int kQHalo = (kMaxBw + 64) / 64;                  // words of halo each side (bw <= kMaxBw)
constexpr int kQWords = kStrip / 64 + 2 * kQHalo;           // 264
constexpr int kQRounds = (kQWords + kWave - 1) / kWave;     // 5

__global__ void __launch_bounds__(256) proc_runs_kernel(ScanParams P) {
    const auto *units = cptr(P.units);
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const int64_t bw = P.bw, gap = 2 * bw + 1;
    const int S = P.S;
    constexpr int64_t kNone = -((int64_t)1 << 40);
    uint32_t cur = 0;
    bool have = false;
    for (uint32_t strip = wave; strip < P.nstrips; strip += nwaves) {
        if (!have) { cur = find_unit(units, P.nunits, strip); have = true; }
        while (strip >= units[cur].strip0 + units[cur].nstrips) ++cur;
        const UnitDesc U = units[cur];
        const uint32_t local = strip - U.strip0;
        const int64_t p0 = 1 + (int64_t)local * kStrip, pend = p0 + kStrip - 1;
        // presence words: word w (lane l, round r: w = 64 r + l - kQHalo) covers p0 + 64 w ..
        uint64_t m[kQRounds];
#pragma unroll
        for (int r = 0; r < kQRounds; ++r) m[r] = 0;
        for (int st = 0; st < U.nstrands; ++st)
            for (int k = 0; k < S; ++k) {
                gu32x4 *t = (gu32x4 *)(track_u8(U, S, st, k) + fbyte(kPadPos + p0 - 1));
#pragma unroll
                for (int r = 0; r < kQRounds; ++r) {
                    const int w = 64 * r + lane - kQHalo;
                    if (w < kQWords - kQHalo) m[r] |= nz_bits64((u32x4)t[w]);
                }
            }
        // previous add before each word (exclusive prefix max of the words'
        // last adds) and next add after it (exclusive suffix min of firsts)
        int64_t prv[kQRounds], nxt[kQRounds];
        int64_t carry = kNone;
#pragma unroll
        for (int r = 0; r < kQRounds; ++r) {
            const int64_t base = p0 + 64 * (64 * r + lane - kQHalo);
            int64_t v = m[r] ? base + 63 - __builtin_clzll(m[r]) : kNone;
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_up((long long)v, d);
                if (lane >= d && o > v) v = o;
            }
            const int64_t ex = __shfl_up((long long)v, 1);
            prv[r] = lane == 0 ? carry : (ex > carry ? ex : carry);
            const int64_t top = __shfl((long long)v, 63);
            carry = top > carry ? top : carry;
        }
        carry = -kNone;  // +inf
#pragma unroll
        for (int r = kQRounds - 1; r >= 0; --r) {
            const int64_t base = p0 + 64 * (64 * r + lane - kQHalo);
            int64_t v = m[r] ? base + __builtin_ctzll(m[r]) : -kNone;
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_down((long long)v, d);
                if (lane + d < 64 && o < v) v = o;
            }
            const int64_t ex = __shfl_down((long long)v, 1);
            nxt[r] = lane == 63 ? carry : (ex < carry ? ex : carry);
            const int64_t bot = __shfl((long long)v, 0);
            carry = bot < carry ? bot : carry;
        }
        // per word: adds that start / end a run (bits at the add positions;
        // the boundary itself sits bw away), and the strip-edge flags
        uint64_t sa[kQRounds], ea[kQRounds];
        bool f0 = false, fl = false;
#pragma unroll
        for (int r = 0; r < kQRounds; ++r) {
            const int64_t base = p0 + 64 * (64 * r + lane - kQHalo);
            sa[r] = ea[r] = 0;
            int64_t prev = prv[r];
            uint64_t mm = m[r];
            while (mm) {
                const int b = __builtin_ctzll(mm);
                mm &= mm - 1;
                const int64_t a = base + b;
                const int64_t nx = mm ? base + __builtin_ctzll(mm) : nxt[r];
                if (prev == kNone || a - prev > gap) sa[r] |= 1ull << b;
                if (nx == -kNone || nx - a > gap) ea[r] |= 1ull << b;
                prev = a;
            }
            f0 |= (m[r] & range_bits(base, p0 - bw, p0 + bw)) != 0;
            fl |= (m[r] & range_bits(base, pend - bw, pend + bw)) != 0;
        }
        const bool F0 = __ballot(f0) != 0, FL = __ballot(fl) != 0;
        // records in position order: starts in (p0, pend], ends in [p0, pend)
        RecList R_{0, 0, kInline};
#pragma unroll
        for (int r = 0; r < kQRounds; ++r) {
            uint64_t live = __ballot(sa[r] != 0);
            while (live) {
                const int l = __builtin_ctzll(live);
                live &= live - 1;
                uint64_t bits = rl_u64(sa[r], l);
                const int64_t base = p0 + 64 * (64 * r + l - kQHalo);
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const int64_t x = base + b - bw;
                    if (x > p0 && x <= pend) rec_start(R_, (uint32_t)x, P, strip, lane);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < kQRounds; ++r) {
            uint64_t live = __ballot(ea[r] != 0);
            while (live) {
                const int l = __builtin_ctzll(live);
                live &= live - 1;
                uint64_t bits = rl_u64(ea[r], l);
                const int64_t base = p0 + 64 * (64 * r + l - kQHalo);
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    const int64_t x = base + b + bw;
                    if (x >= p0 && x < pend) rec_end(R_, (uint32_t)x, 0u, -__builtin_inf(), P, strip, lane);
                }
            }
        }
        const uint64_t info = (uint64_t)R_.ns | ((uint64_t)R_.ne << 16) | ((uint64_t)F0 << 32) |
                              ((uint64_t)FL << 33) | ((uint64_t)(local == 0) << 34) |
                              ((uint64_t)(local + 1 == U.nstrips) << 35) | ((uint64_t)(R_.slot != kInline) << 36);
        if (lane == 0) P.strip_info[strip] = info;
    }
}

// K1q's fallback test: a unit with an add at a position <= bw + 1 starts
// processing at position 1 (a single step, or the misaligned window of quirk
// Q1): the host then replays the whole buffer.  One block per unit.
__global__ void __launch_bounds__(256) q11_head_kernel(const UnitDesc *units, int S, int bw, uint32_t *flag) {
    const UnitDesc U = units[blockIdx.x];
    bool any = false;
    for (int st = 0; st < U.nstrands; ++st)
        for (int k = 0; k < S; ++k)
            for (int p = 1 + (int)threadIdx.x; p <= bw + 1 && p <= (int)U.len; p += blockDim.x)
                any |= fld_at(track_u8(U, S, st, k), p) != 0u;
    if (__syncthreads_or(any) && threadIdx.x == 0) flag[blockIdx.x] = 1u;
}

// K1x: the K1a waves' stash counts -> xref (stash indices of the listed
// entries, every front entry first) and the totals in xcount.  One block:
// thread t owns K1a waves [t*per, (t+1)*per).
__global__ void __launch_bounds__(1024) xref_kernel(const uint32_t *__restrict__ xwcount, uint32_t nw,
                                                    uint32_t xcap, uint32_t *__restrict__ xref,
                                                    uint32_t *__restrict__ xcount) {
    __shared__ uint64_t sc[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nw + 1023) / 1024;
    const uint32_t w0 = t * per, w1 = w0 + per < nw ? w0 + per : nw;
    uint64_t mine = 0;  // front count | back count << 32 (totals < 2^32)
    for (uint32_t w = w0; w < w1; ++w) mine += (uint64_t)xwcount[2 * w] | ((uint64_t)xwcount[2 * w + 1] << 32);
    sc[t] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan
        const uint64_t v = t >= o ? sc[t - o] : 0;
        __syncthreads();
        sc[t] += v;
        __syncthreads();
    }
    const uint64_t tot = sc[1023];
    const uint32_t nf = (uint32_t)tot;
    uint32_t of = (uint32_t)(sc[t] - mine), ob = nf + (uint32_t)((sc[t] - mine) >> 32);
    for (uint32_t w = w0; w < w1; ++w) {
        const uint32_t a = xwcount[2 * w], b = xwcount[2 * w + 1];
        for (uint32_t k = 0; k < a; ++k) xref[of++] = w * xcap + k;
        for (uint32_t k = 0; k < b; ++k) xref[ob++] = w * xcap + xcap - 1 - k;
    }
    if (t == 0) {
        xcount[0] = nf;
        xcount[1] = (uint32_t)(tot >> 32);
    }
}

// ------------------------------------------------------------------------
// K2: segmentation in two launches (no library scan, no host round trip).
// Per-strip (starts, ends) counts are packed into one uint64 (starts in the
// low, ends in the high half; totals stay < 2^32, so packed sums never carry).
// ------------------------------------------------------------------------
constexpr int kSegBlock = 256;

// packed count of strip i: interior runs plus the run that starts at the
// strip's first position / ends at its last one when the neighbour strip
// (same unit) does not continue it
__device__ __forceinline__ uint64_t seg_count(const uint64_t *__restrict__ info, uint32_t i) {
    const uint64_t v = info[i];
    const uint32_t prev_last = si_bit(v, 34) ? 0u : si_bit(info[i - 1], 33);
    const uint32_t next_first = si_bit(v, 35) ? 0u : si_bit(info[i + 1], 32);
    const uint32_t xs = si_bit(v, 32) & (prev_last ^ 1u);
    const uint32_t xe = si_bit(v, 33) & (next_first ^ 1u);
    return (uint64_t)(si_starts(v) + xs) | ((uint64_t)(si_ends(v) + xe) << 32);
}

__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, uint64_t *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((long long)v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// K2a: per-strip counts and one packed total per 256 strips
__device__ __forceinline__ void seg_count_block(const uint64_t *__restrict__ info, uint64_t *__restrict__ cnt,
                                                uint64_t *__restrict__ bsum, uint32_t n) {
    __shared__ uint64_t red[4];
    const uint32_t i = blockIdx.x * kSegBlock + threadIdx.x;
    uint64_t c = 0;
    if (i < n) {
        c = seg_count(info, i);
        cnt[i] = c;
    }
    const uint64_t t = block_sum_u64(c, red);
    if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

// K2b: each block adds up the totals of the blocks before it, scans its own
// 256 counts and compacts its run boundaries into the region lists; the last
// block publishes the region count (status[0] = regions, status[1] = spilled
// strips, status[2] = start/end mismatch) and re-arms the pass counters
__global__ void __launch_bounds__(kSegBlock) seg_compact_kernel(
    const UnitDesc *units, uint32_t nunits, const uint64_t *__restrict__ info,
    const uint64_t *__restrict__ cnt, const uint64_t *__restrict__ bsum, const uint32_t *__restrict__ rec,
    const uint32_t *__restrict__ ovf_rec, uint32_t ovf_cap, uint32_t *__restrict__ starts,
    uint32_t *__restrict__ ends, uint32_t *__restrict__ reg_unit, uint32_t *__restrict__ peak_pos,
    double *__restrict__ peak_val, uint32_t n, uint64_t cap, uint32_t *ovf_count, uint32_t *xcount,
    uint64_t *nreg, unsigned long long *status, unsigned long long *target_hdr) {
    __shared__ uint64_t red[4];
    __shared__ uint64_t wsum[4];
    uint64_t part = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kSegBlock) part += bsum[j];
    const uint64_t base = block_sum_u64(part, red);
    const uint32_t i = blockIdx.x * kSegBlock + threadIdx.x;
    const uint64_t c = i < n ? cnt[i] : 0;
    // block exclusive scan: wave inclusive scan, then the waves before
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = (uint64_t)__shfl_up((long long)inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0;
    for (int k = 0; k < w; ++k) before += wsum[k];
    const uint64_t o = base + before + inc - c;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kSegBlock - 1) {
        const uint64_t t = o + c;
        const uint64_t nst = t & 0xFFFFFFFFull, nen = t >> 32;
        const uint32_t ovf = *ovf_count;
        // a pass whose record areas overflowed left gaps in the region lists:
        // K3 must see no region at all (the host grows the areas and reruns)
        const bool valid = nst <= cap && nst == nen && ovf <= ovf_cap;
        *nreg = valid ? nst : 0;
        status[0] = nst;
        status[1] = ovf;
        status[2] = nst != nen;
        if (target_hdr) *target_hdr = valid ? nst : 0;  // caller's record buffer (up_set_record_target)
        *ovf_count = 0u;                    // K1b has consumed the work list
        xcount[0] = 0u;
        xcount[1] = 0u;
    }
    if (c == 0) return;
    const uint64_t v = info[i];
    const uint32_t ns = (uint32_t)c, ne = (uint32_t)(c >> 32);
    const uint32_t xs = ns - si_starts(v), xe = ne - si_ends(v);
    uint32_t os = (uint32_t)o, oe = (uint32_t)(o >> 32);
    const uint32_t u = find_unit(units, nunits, i);
    const int64_t p0 = 1 + (int64_t)(i - units[u].strip0) * kStrip;
    const uint32_t *src = rec + (uint64_t)i * kRecStride;
    uint32_t half = kCap;
    if (si_bit(v, 36)) {
        const uint32_t slot = src[0];
        if (slot >= ovf_cap) return;  // host grows the area and reruns
        src = ovf_rec + (uint64_t)slot * kOvfStride;
        half = kOvfHalf;
    }
    const uint32_t *spk = src + 2 * half;
    const double *spv = (const double *)(src + 4 * half);
    if (os + ns > cap || oe + ne > cap) return;  // host grows the areas and reruns
    if (xs) { starts[os] = (uint32_t)p0; reg_unit[os] = u; ++os; }
    for (uint32_t k = 0; k < si_starts(v); ++k) { starts[os] = src[k]; reg_unit[os] = u; ++os; }
    for (uint32_t k = 0; k < si_ends(v); ++k) {
        peak_pos[oe] = spk[k];
        peak_val[oe] = spv[k];
        ends[oe++] = src[half + k];
    }
    if (xe) { peak_pos[oe] = 0; peak_val[oe] = 0.0; ends[oe++] = (uint32_t)(p0 + kStrip - 1); }
}

// ---- the per-dataset index (kernels.h: chunk-sum planes, pooled planes,
// pooled count tracks), built for many units in one launch each.  Work item
// i of the launch belongs to list entry k with off[k] <= i < off[k + 1]
// (off: exclusive prefix of the entries' item counts, off[n] = total).
// (a grid-stride loop's items only grow: the entry advances from the
// previous one, a binary search only for the thread's first item)
__device__ __forceinline__ uint32_t list_entry(const uint64_t *off, uint32_t n, uint64_t i, uint32_t &k) {
    if (k == ~0u) {
        uint32_t lo = 0, hi = n;  // the last k with off[k] <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= i) lo = mid; else hi = mid;
        }
        k = lo;
    }
    while (k + 1 < n && off[k + 1] <= i) ++k;
    return k;
}

// chunk-sum planes: one item per 4 chunks (one 16-byte load of a track, one
// dword of its plane) of every track of the listed units; escaped fields at
// their overflow counts, each chunk saturated at 255
__global__ void __launch_bounds__(256) csum_units_kernel(const UnitDesc *units, const uint32_t *list,
                                                         const uint64_t *off, uint32_t n, int S) {
    const uint64_t total = off[n];
    uint32_t kc = ~0u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = list_entry(off, n, i, kc);
        const UnitDesc U = units[list[k]];
        const uint64_t nq = U.stride / 16;  // items per track
        const uint64_t r = i - off[k];
        const uint32_t t = (uint32_t)(r / nq);
        const uint64_t q = r - (uint64_t)t * nq;
        const uint32_t ntr = (uint32_t)U.nstrands * (uint32_t)S;
        const u32x4 v = *(const u32x4 *)((const uint8_t *)U.base + (uint64_t)t * U.stride + 16 * q);
        const uint32_t d[4] = {v.x, v.y, v.z, v.w};
        uint32_t out = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint32_t sum = fsum32(d[c], 0u);  // an escaped field counts kEsc here
            uint32_t e = fbig32(d[c]);
            while (e && sum < 255u) {
                const int b = __builtin_ctz(e);
                e &= e - 1u;
                const int64_t p = (int64_t)(16 * (4 * q + c)) + b / kTB - kPadPos + 1;  // the field's position
                const uint32_t cnt = ovf_lookup(U, t, (uint32_t)p);
                sum = sum - kEsc + (cnt < 255u ? cnt : 255u);
            }
            out |= (sum < 255u ? sum : 255u) << (8 * c);
        }
        uint8_t *plane = (uint8_t *)U.base + (uint64_t)ntr * U.stride;
        *(uint32_t *)(plane + (uint64_t)t * (U.stride / 4) + 4 * q) = out;
    }
}

// pooled planes: one item per 4 chunks of each listed unit -- per chunk the
// weighted sum of the non-control samples' planes over the unit's strands
// (w <= 4096: no wrap), saturated at 255
__global__ void __launch_bounds__(256) pool_units_kernel(const UnitDesc *units, const uint32_t *list,
                                                         const uint64_t *off, uint32_t n, int S, int nnc,
                                                         const int32_t *nc, const uint32_t *w) {
    const uint64_t total = off[n];
    uint32_t kc = ~0u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = list_entry(off, n, i, kc);
        const UnitDesc U = units[list[k]];
        const uint64_t nd = U.stride / 4;  // plane bytes per track
        const uint64_t q = i - off[k];
        const uint8_t *planes = (const uint8_t *)U.base + (uint64_t)U.nstrands * S * U.stride;
        uint32_t s[4] = {0u, 0u, 0u, 0u};
        for (int st = 0; st < U.nstrands; ++st)
            for (int j = 0; j < nnc; ++j) {
                const uint32_t b = *(const uint32_t *)(planes + ((uint64_t)st * S + nc[j]) * nd + 4 * q);
                if (!b) continue;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t v = s[c] + w[j] * ((b >> (8 * c)) & 0xFFu);
                    s[c] = v < 255u ? v : 255u;
                }
            }
        uint8_t *pooled = (uint8_t *)planes + (uint64_t)U.nstrands * S * nd;
        *(uint32_t *)(pooled + 4 * q) = s[0] | (s[1] << 8) | (s[2] << 16) | (s[3] << 24);
    }
}

// pooled count tracks (UnitDesc::pct): one item per track dword (16
// positions) and strand of each listed unit, the pooled samples' fields
// summed (escapes at their counts), saturated at 255; pct: the unit's
// allocation (listed units only)
__global__ void __launch_bounds__(256) pct_units_kernel(const UnitDesc *units, const uint32_t *list,
                                                        const uint64_t *off, uint32_t n, int S, int nnc,
                                                        const int32_t *nc, uint8_t *const *pct) {
    const uint64_t total = off[n];
    uint32_t kc = ~0u;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = list_entry(off, n, i, kc);
        const UnitDesc U = units[list[k]];
        const uint64_t nd = U.stride / 4;  // dwords per track
        const uint64_t r = i - off[k];
        const int st = (int)(r / nd);
        const uint64_t j = r - (uint64_t)st * nd;
        uint32_t sum[16];
#pragma unroll
        for (int f = 0; f < 16; ++f) sum[f] = 0;
        for (int m = 0; m < nnc; ++m) {
            const uint32_t d = ((const uint32_t *)((const uint8_t *)U.base + ((uint64_t)st * S + nc[m]) * U.stride))[j];
            if (!d) continue;
#pragma unroll
            for (int f = 0; f < 16; ++f) {
                uint32_t v = (d >> (2 * f)) & 3u;
                if (v == kEsc) {
                    const int64_t p = (int64_t)(16 * j) + f - kPadPos + 1;
                    v = ovf_lookup(U, (uint32_t)(st * S + nc[m]), (uint32_t)p);
                }
                sum[f] += v;
            }
        }
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            o[q] = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) o[q] |= (sum[4 * q + b] < 255u ? sum[4 * q + b] : 255u) << (8 * b);
        }
        uint4 *dst = (uint4 *)(pct[k] + (uint64_t)st * (4 * U.stride) + 16 * j);
        *dst = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// per-unit last add (the last position whose pooled count is nonzero): one
// wave per strip finds its highest nonzero field over the pooled tracks and
// folds it into the unit's slot with atomicMax (out zeroed by the caller)
__device__ __forceinline__ uint32_t top_fld(uint32_t x) {  // index of the highest nonzero field
    return (uint32_t)(31 - __builtin_clz(x)) / (uint32_t)kTB;
}

__global__ void __launch_bounds__(256) unit_last_kernel(const UnitDesc *units, uint32_t nunits,
                                                        uint32_t nstrips, int S, int nnc,
                                                        const int32_t *nc, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells the compiler, so the
    // strip / unit / work-list indices derived from it live in SGPRs and the
    // unit table is read with scalar loads (vector loads of it cost a
    // dependent round trip behind the streaming loads on every strip)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t strip = wave; strip < nstrips; strip += nwaves) {
        const uint32_t u = find_unit(units, nunits, strip);
        const UnitDesc U = units[u];
        const int64_t p0 = 1 + (int64_t)(strip - U.strip0) * kStrip;
        uint32_t best = 0;
        for (int st = 0; st < U.nstrands; ++st)
            for (int k = 0; k < nnc; ++k) {
                gu32x4 *t = (gu32x4 *)(track_u8(U, S, st, nc[k]) + fbyte(kPadPos + p0 - 1));
                constexpr int PD = 4 * kPerByte;  // positions per dword
#pragma unroll 4
                for (int bk = 0; bk < kStripBytes / (kWave * 16); ++bk) {
                    const u32x4 v = __builtin_nontemporal_load(t + 64 * bk + lane);
                    const int64_t q = p0 + 64 * 4 * PD * bk + 4 * PD * lane;  // the lane's first position
                    uint32_t hi = 0;
                    if (v.x) hi = (uint32_t)q + top_fld(v.x);
                    if (v.y) hi = (uint32_t)q + PD + top_fld(v.y);
                    if (v.z) hi = (uint32_t)q + 2 * PD + top_fld(v.z);
                    if (v.w) hi = (uint32_t)q + 3 * PD + top_fld(v.w);
                    best = hi > best ? hi : best;
                }
            }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t ob = (uint32_t)__shfl_xor((int)best, o);
            best = ob > best ? ob : best;
        }
        if (lane == 0 && best) atomicMax(&out[u], best);
    }
}

#endif  // UPK_NH_TU

// ------------------------------------------------------------------------
// K3: region statistics, one wave per region (grid-stride).
// ------------------------------------------------------------------------


// pooled counts of the 2NH+1 words around block start x0 for one strand
template <int NH, int POOL>
__device__ __forceinline__ void region_words(WinT<POOL> (&cs)[2 * NH + 1], uint64_t (&hm)[2 * NH + 1],
                                             const UnitDesc &U, int strand, int64_t x0, int lane,
                                             const StatParams &P) {
    load_words<2 * NH + 1, POOL>(cs, U, P.S, strand, x0 - 64 * NH, lane, P.nnc, P.nc, P.coef);
#pragma unroll
    for (int w = 0; w < 2 * NH + 1; ++w) hm[w] = __ballot(nz(cs[w]));
}

// sum of one track's counts over positions [left, right]: the chunk-sum plane
// for whole chunks (a saturated 255 and the two partial chunks at the ends
// from the track's dword, escapes at their overflow counts)
// (planes false: the pass runs without the index -- every chunk from its dword)
__device__ __forceinline__ uint32_t track_range_sum(const UnitDesc &U, int S, int st, int smp, uint32_t left,
                                                    uint32_t right, bool planes) {
    gu32 *tw = (gu32 *)track_u8(U, S, st, smp);
    gu8 *pl = plane_u8(U, S, st, smp);
    const uint32_t track = (uint32_t)(st * S + smp);
    const int64_t n0 = kPadPos + (int64_t)left - 1, n1 = kPadPos + (int64_t)right - 1;
    const int64_t j0 = n0 >> 4, j1 = n1 >> 4;
    auto dsum = [&](int64_t j, int f0, int f1) -> uint32_t {  // fields f0..f1 of dword j
        const uint32_t mask = (f1 - f0 == 15) ? ~0u : (((1u << (2 * (f1 - f0 + 1))) - 1u) << (2 * f0));
        const uint32_t d = tw[j] & mask;
        uint32_t sum = fsum32(d, 0u);  // an escaped field counts kEsc here
        uint32_t e = fbig32(d);
        while (e) {
            const int b = __builtin_ctz(e);
            e &= e - 1u;
            const int64_t p = 16 * j + b / 2 - kPadPos + 1;
            sum += ovf_lookup(U, track, (uint32_t)p) - kEsc;
        }
        return sum;
    };
    if (j0 == j1) return dsum(j0, (int)(n0 & 15), (int)(n1 & 15));
    uint32_t sum = dsum(j0, (int)(n0 & 15), 15) + dsum(j1, 0, (int)(n1 & 15));
#pragma unroll 4
    for (int64_t j = j0 + 1; j < j1; ++j) {
        const uint32_t b = planes ? (uint32_t)pl[j] : 255u;
        sum += b == 255u ? dsum(j, 0, 15) : b;
    }
    return sum;
}

// exptSums[s] += t (t wave-uniform): up to 256 samples in registers -- lane
// s % 64, slot s / 64 -- beyond that (esl != null) in the wave's LDS row of
// S words (the reference's nExpt_ is a UShort, misc/peakcall.hpp:49)
__device__ __forceinline__ void add_es(uint32_t (&esum)[4], uint32_t *esl, int s, uint32_t t, int lane) {
    if (esl) {
        if (lane == 0) esl[s] += t;
        return;
    }
    if (lane == (s & 63)) {
        const int slot = s >> 6;
        esum[0] += slot == 0 ? t : 0u;
        esum[1] += slot == 1 ? t : 0u;
        esum[2] += slot == 2 ? t : 0u;
        esum[3] += slot == 3 ? t : 0u;
    }
}

// exptSums of the non-control samples over a region: every tag of a
// non-control sample is a pooled hit, so its exptSum is its track's range
// sum (one lane per (strand, sample) track; sc: 256 words of the wave's LDS,
// or the wave's exptSums row esl itself beyond 256 samples)
template <bool NONDIR>
__device__ __forceinline__ void nc_range_sums(uint32_t (&esum)[4], uint32_t *esl, const UnitDesc &U,
                                              const StatParams &P, uint32_t left, uint32_t right, int lane,
                                              uint32_t *sc) {
    const int S = P.S, nnc = P.nnc;
    constexpr int NSTR = NONDIR ? 2 : 1;
    if (esl) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // lane 0's row updates are visible
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int t = lane; t < nnc * NSTR; t += 64) {
            const int st = t >= nnc ? 1 : 0;
            const int smp = P.nc[t - st * nnc];
            atomicAdd(&esl[smp], track_range_sum(U, S, st, smp, left, right, P.planes != 0));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        return;
    }
    __builtin_amdgcn_wave_barrier();  // earlier readers of the area are done
    for (int i = lane; i < S; i += 64) sc[i] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = lane; t < nnc * NSTR; t += 64) {
        const int st = t >= nnc ? 1 : 0;
        const int smp = P.nc[t - st * nnc];
        atomicAdd(&sc[smp], track_range_sum(U, S, st, smp, left, right, P.planes != 0));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int smp = 64 * q + lane;
        if (smp < S && !P.is_control[smp]) esum[q] += sc[smp];
    }
    __builtin_amdgcn_wave_barrier();  // the area is reused
}

// K3's occupancy: 5 waves per EU, i.e. <= 96 VGPRs (one directional
// sample: a 40-byte spill), so two K3 waves fit beside K1a's three per SIMD.
// Same-box A/B (profiles/r04/k1b_dead/, k3_all/): configs[1] K3 alone 0.160
// -> 0.144 ms, step +1.2 % over three rounds; configs[2] K3 0.54 -> 0.49 ms,
// step +4.3 % over two; configs[4] replicates unchanged
#ifndef UPK_K3_WPE
#define UPK_K3_WPE 5
#endif
template <int NH, int POOL, bool NONDIR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UPK_K3_WPE))) stats_kernel(StatParams P) {
    extern __shared__ double lds_[];
    const int bw = P.bw;
    const double *ktab = load_ktab(lds_, P.kern, bw);
    constexpr int NWT = 2 * NH + 1;
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane tells the compiler, so the
    // strip / unit / work-list indices derived from it live in SGPRs and the
    // unit table is read with scalar loads (vector loads of it cost a
    // dependent round trip behind the streaming loads on every strip)
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const uint64_t nreg = *P.nreg < P.cap ? *P.nreg : P.cap;
    uint64_t wm[2 * NH + 1];
#pragma unroll
    for (int d = -NH; d <= NH; ++d) wm[d + NH] = win_mask(d, bw);
    const int S = P.S;  // <= kMaxSamples (checked by the host)
    // exptSums beyond 256 samples: one row of S words per wave after the
    // terms areas (dynamic LDS sized by the host, dispatch_stats)
    uint32_t *esl = S > 256 ? (uint32_t *)((double2 *)((uint32_t *)(lds_ + kKTab) + 4 * kStatCache * 64) + 4 * 64) +
                                  (threadIdx.x >> 6) * S
                            : nullptr;
    // several samples, integer pooling: the non-control samples' exptSums are
    // range sums of their chunk-sum planes (nc_range_sums), the pooled count
    // of a hit is the window word's own value
    constexpr bool kRS = kTB == 2 && POOL != 2;

    // per-wave cache of the pass-1 hit totals pc (pass 2 reads them back)
    uint32_t *pcache = (uint32_t *)(lds_ + kKTab) + (threadIdx.x >> 6) * (kStatCache * 64);
    double2 *terms = (double2 *)((uint32_t *)(lds_ + kKTab) + 4 * kStatCache * 64) + (threadIdx.x >> 6) * 64;
    // this wave's slab of (f, r) per region position for the correlation
    double2 *cslab = (NONDIR && P.want_corr && P.corr_scratch)
                         ? (double2 *)P.corr_scratch + (uint64_t)wave * P.corr_cap : nullptr;

    // K1 saw the whole run: its peak is known and, unless the strand
    // correlation is wanted, no score is needed here -- only the counts
    const bool known = P.peak_pos != nullptr && !(NONDIR && P.want_corr);
    // Region descriptors (start, end, unit, peak position, peak value) come
    // one region ahead: lanes 0..5 read the next region's six words with one
    // vector load at the top of an iteration, and with one pooled directional
    // sample the next region's count bytes are fetched before this region's
    // kurtosis pass, so the loads of region i+1 overlap the work of region i
    // (a wave holds ~10 regions; their dependent load chains were the cost).
    constexpr bool kPrefetch = POOL == 0 && !NONDIR;
    auto desc_load = [&](uint64_t r) -> uint32_t {
        if (lane >= (known ? 6 : 3)) return 0u;
        const uint32_t *src = lane == 0   ? P.starts + r
                              : lane == 1 ? P.ends + r
                              : lane == 2 ? P.reg_unit + r
                              : lane == 3 ? P.peak_pos + r
                                          : (const uint32_t *)(P.peak_val + r) + (lane - 4);
        return *src;
    };
    uint32_t dsc = wave < nreg ? desc_load(wave) : 0u;
    bool pre_ok = false;  // praw holds the count bytes of region ri
    uint32_t praw[kPrefetch ? kStatCache : 1];
    bool pk_pre = false;  // pkraw holds the bytes of the window around pk_pos (Q keys)
    uint32_t pk_pos = 0, pkraw[kPrefetch ? 2 * NH : 1];
    for (uint64_t ri = wave; ri < nreg; ri += nwaves) {
        const uint32_t left = rl_u(dsc, 0), right = rl_u(dsc, 1), u = rl_u(dsc, 2);
        const uint64_t rn = ri + nwaves;
        const uint32_t dsc_n = rn < nreg ? desc_load(rn) : 0u;
        const UnitDesc U = P.units[u];
        uint32_t esum[4] = {0, 0, 0, 0};  // exptSums[s] lives in lane s%64, slot s/64 (or esl)
        if (esl) {
            __builtin_amdgcn_wave_barrier();  // the previous region's reads are done
            for (int i = lane; i < S; i += 64) esl[i] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        uint32_t esum1 = 0;               // S == 1: lane-local partial of exptSums[0]

        uint32_t cnt_acc = 0, sum_acc = 0;
        double best = 0.0;
        int64_t best_x = -1;
        double sf = 0.0, sr = 0.0;  // sequential sums of f and r (corr means)
        // ---- pass 1: scores, peak, exptSums, kurtosis first moments ----
        // POOL 0: raw bytes of the next 64-position window are fetched while
        // the current one is scored (escapes resolved at use)
        uint32_t nf[NWT], nr[NONDIR ? NWT : 1];
        auto fetch_raw = [&](uint32_t (&dst)[NWT], int strand, int64_t x0) {
            const int64_t n0 = kPadPos + (x0 - 64 * NH) - 1 + lane;
            gu8 *t = track_u8(U, S, strand, P.nc[0]) + fbyte(n0);
            const uint32_t sh = fshift(n0);
#pragma unroll
            for (int w = 0; w < NWT; ++w) dst[w] = ((uint32_t)t[kWordBytes * w] >> sh) & kTMask;
        };
        uint32_t kpos = 0;
        double kval = 0.0;
        if (known) {
            kpos = rl_u(dsc, 3);
            kval = __longlong_as_double((long long)(((uint64_t)rl_u(dsc, 5) << 32) | rl_u(dsc, 4)));
            if (kpos == 0) {
                // the run crossed a strip edge: first maximum over its parts,
                // in position order -- the part of the run open at a strip's
                // first position that closes inside it, else the part open at
                // the strip's last position (from the run start or the strip's
                // first position)
                const uint32_t sa = U.strip0 + (left - 1) / kStrip, sb = U.strip0 + (right - 1) / kStrip;
                for (uint32_t s = sa; s <= sb; ++s) {
                    const uint32_t sp0 = 1 + (s - U.strip0) * kStrip;
                    const bool pre = (s > sa || left == sp0) && s == sb && right < sp0 + kStrip - 1;
                    const uint64_t *e = P.spk + 4ull * s + (pre ? 0 : 2);
                    const double v = __longlong_as_double((long long)e[0]);
                    if (P.qmode) {  // Q keys: equal Q in two parts is a tie too
                        const double fv = __builtin_floor(v), fk = __builtin_floor(kval);
                        if (s == sa || fv > fk) {
                            kval = v;
                            kpos = (uint32_t)e[1];
                        } else if (fv == fk) {
                            kval = fk + 0.5;
                        }
                    } else if (s == sa || v > kval) {
                        kval = v;
                        kpos = (uint32_t)e[1];
                    }
                }
            }
        }
        // Q keys (K1b, ScanParams::qmode) give the peak position; a key
        // marked +0.5 (the largest Q at two positions) leaves the first
        // maximum to the FP64 scores of this region's KDE below
        const bool kn = known && !(P.qmode && kval != __builtin_floor(kval));
        // the peak's FP64 score: the pooled counts of its window (2NH words
        // from kpos - bw, lane = offset t), fetched now and summed after the
        // region's counts
        // (several pooled samples without coefficients: their pooled count
        // words, one byte each from the pooled count track)
        constexpr int kPK = POOL != 2 ? 2 * NH : 1;
        WinT<POOL> pkf[kPK], pkr[NONDIR ? kPK : 1];
        if (POOL != 2 && kn && P.qmode) {
            if (kPrefetch && pk_pre && pk_pos == kpos) {  // fetched during the previous region
                const uint32_t sh = fshift(kPadPos + (int64_t)kpos - bw - 1 + lane);
                uint32_t c[kPrefetch ? 2 * NH : 1];
#pragma unroll
                for (int w = 0; w < (kPrefetch ? 2 * NH : 1); ++w) c[w] = (pkraw[w] >> sh) & kTMask;
                resolve_escapes<kPrefetch ? 2 * NH : 1>(c, U, (uint32_t)P.nc[0], (int64_t)kpos - bw, lane);
#pragma unroll
                for (int w = 0; w < (kPrefetch ? 2 * NH : 1); ++w) pkf[w] = c[w];
            } else {
                load_words<kPK, POOL>(pkf, U, S, 0, (int64_t)kpos - bw, lane, P.nnc, P.nc, P.coef);
            }
            if constexpr (NONDIR)
                load_words<kPK, POOL>(pkr, U, S, 1, (int64_t)kpos - bw, lane, P.nnc, P.nc, P.coef);
        }
        int blk = 0;
        bool counted = false, staged = false;
        if constexpr (POOL == 0) {
            // one pooled sample: the region's count bytes (<= kStatCache
            // words) are fetched with all loads in flight at once, then
            // scored; escapes resolved at use
            const int nw = (int)((right - left) / 64u) + 1;
            if (kn && S == 1 && nw <= kStatCache) {
                best = kval;
                best_x = kpos;
                const int64_t n0 = kPadPos + (int64_t)left - 1 + lane;
                const uint32_t sh = fshift(n0);
                gu8 *t0 = track_u8(U, S, 0, P.nc[0]) + fbyte(n0);
                uint32_t r0[kStatCache], r1[NONDIR ? kStatCache : 1];
                if (kPrefetch && pre_ok) {
#pragma unroll
                    for (int w = 0; w < kStatCache; ++w) r0[w] = praw[kPrefetch ? w : 0];
                } else {
#pragma unroll
                    for (int w = 0; w < kStatCache; ++w) r0[w] = w < nw ? t0[kWordBytes * w] : 0u;
                }
                if constexpr (NONDIR) {
                    gu8 *t1 = track_u8(U, S, 1, P.nc[0]) + fbyte(n0);
#pragma unroll
                    for (int w = 0; w < kStatCache; ++w) r1[w] = w < nw ? t1[kWordBytes * w] : 0u;
                }
#pragma unroll
                for (int w = 0; w < kStatCache; ++w) {
                    r0[w] = (r0[w] >> sh) & kTMask;
                    if constexpr (NONDIR) r1[w] = (r1[w] >> sh) & kTMask;
                }
                resolve_escapes<kStatCache>(r0, U, (uint32_t)P.nc[0], (int64_t)left, lane);
                if constexpr (NONDIR) resolve_escapes<kStatCache>(r1, U, (uint32_t)(S + P.nc[0]), (int64_t)left, lane);
#pragma unroll
                for (int w = 0; w < kStatCache; ++w) {
                    if (w >= nw) break;
                    const int64_t x = (int64_t)left + 64 * w + lane;
                    const bool valid = x <= (int64_t)right;
                    uint32_t pc = valid ? r0[w] : 0u;
                    if constexpr (NONDIR) pc += valid ? r1[w] : 0u;
                    esum1 += pc;
                    pcache[64 * w + lane] = pc;
                    cnt_acc += pc;
                    sum_acc += pc * (uint32_t)(uint16_t)(x - left);
                }
                blk = nw;
                counted = true;
            }
        }
        // (2-bit tracks only: a 64-position block spans at most 32 bytes
        // from its 16-byte-aligned base only at 4 positions per byte; the
        // 4-bit A/B build takes the per-sample path)
        static_assert(kTB == 2 || kTB == 4, "track layout");
        if constexpr (POOL != 2 && kTB == 2) {
            // several samples (and at most 32 (strand, sample) tracks): each
            // 64-position block's bytes of every track come with one wave
            // load (lane l: track l/2, 16-byte piece l%2 of the 32 bytes
            // covering the block), staged through this wave's terms area and
            // read back as lane = position; the next block's load is in
            // flight meanwhile.  (Per sample, pooled fetch then count_at, the
            // block cost S + nnc dependent round trips.)
            constexpr int NSTR = NONDIR ? 2 : 1;
            if (kn && !counted && S > 1 && S * NSTR <= 32) {
                best = kval;
                best_x = kpos;
                const int jt = lane >> 1;
                const bool tl = jt < S * NSTR;
                gu8 *tb = track_u8(U, S, tl ? jt / S : 0, tl ? jt % S : 0);
                auto bload = [&](int64_t x0) -> u32x4 {
                    u32x4 r = {0u, 0u, 0u, 0u};
                    if (tl) r = ((gu32x4 *)(tb + (fbyte(kPadPos + x0 - 1) & ~(int64_t)15)))[lane & 1];
                    return r;
                };
                uint8_t *stg = (uint8_t *)terms;
                u32x4 nv = bload(left);
                for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64, ++blk) {
                    const int64_t x = x0 + lane;
                    const bool valid = x <= (int64_t)right;
                    const u32x4 cv = nv;
                    if (x0 + 64 <= (int64_t)right) nv = bload(x0 + 64);
                    __builtin_amdgcn_wave_barrier();  // the previous block's reads are done
                    *(u32x4 *)(stg + 16 * lane) = cv;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    const int64_t n0 = kPadPos + x - 1;
                    const uint32_t off = (uint32_t)(fbyte(n0) - (fbyte(kPadPos + x0 - 1) & ~(int64_t)15));
                    const uint32_t sh = fshift(n0);
                    auto fld = [&](int j) -> uint32_t {  // track j = strand * S + sample
                        const uint32_t f = ((uint32_t)stg[32 * j + off] >> sh) & kTMask;
                        return (f == kEsc && valid) ? ovf_lookup(U, (uint32_t)j, (uint32_t)x) : f;
                    };
                    uint32_t pf = 0, pr = 0;  // pooled counts (their sum is exact: host bound)
                    for (int k = 0; k < P.nnc; ++k) {
                        pf += fld(P.nc[k]);
                        if constexpr (NONDIR) pr += fld(S + P.nc[k]);
                    }
                    const bool h0 = valid && pf != 0u;
                    const bool h1 = NONDIR && valid && pr != 0u;
                    uint32_t pc = 0;
                    // (every sample from the stage: cheaper here than the
                    // plane range sums -- configs[3] K3 0.53 vs 0.73 ms)
                    for (int s = 0; s < S; ++s) {
                        uint32_t c = h0 ? fld(s) : 0u;
                        if constexpr (NONDIR) c += h1 ? fld(S + s) : 0u;
                        pc += c;
                        const uint32_t t = wave_sum_u32(c);
                        add_es(esum, esl, s, t, lane);
                    }
                    if (blk < kStatCache) pcache[64 * blk + lane] = pc;
                    cnt_acc += pc;
                    sum_acc += pc * (uint32_t)(uint16_t)(x - left);
                }
                __builtin_amdgcn_wave_barrier();  // terms reused below
                counted = true;
                staged = true;
            }
        }
        if (kn && !counted) {
            best = kval;
            best_x = kpos;
            for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64, ++blk) {
                const int64_t x = x0 + lane;
                const bool valid = x <= (int64_t)right;
                WinT<POOL> c0[1], c1[1];
                load_words<1, POOL>(c0, U, S, 0, x0, lane, P.nnc, P.nc, P.coef);
                if constexpr (NONDIR) load_words<1, POOL>(c1, U, S, 1, x0, lane, P.nnc, P.nc, P.coef);
                const bool h0 = valid && nz(c0[0]);
                const bool h1 = NONDIR && valid && nz(c1[0]);
                uint32_t pc = 0;
                if (POOL == 0 && S == 1) {
                    if (h0) pc += (uint32_t)c0[0];
                    if (h1) pc += (uint32_t)c1[0];
                    esum1 += pc;
                } else if (kRS) {  // (as in the scoring loop below)
                    if (h0) pc += (uint32_t)c0[0];
                    if (h1) pc += (uint32_t)c1[0];
                    for (int s = 0; s < S && P.nnc < S; ++s) {
                        if (!P.is_control[s]) continue;
                        uint32_t c = 0;
                        if (h0) c += count_at(U, S, 0, s, x);
                        if (h1) c += count_at(U, S, 1, s, x);
                        pc += c;
                        const uint32_t t = wave_sum_u32(c);
                        add_es(esum, esl, s, t, lane);
                    }
                } else {
                    for (int s = 0; s < S; ++s) {
                        uint32_t c = 0;
                        if (h0) c += count_at(U, S, 0, s, x);
                        if (h1) c += count_at(U, S, 1, s, x);
                        pc += c;
                        const uint32_t t = wave_sum_u32(c);
                        add_es(esum, esl, s, t, lane);
                    }
                }
                if (blk < kStatCache) pcache[64 * blk + lane] = pc;
                cnt_acc += pc;
                sum_acc += pc * (uint32_t)(uint16_t)(x - left);
            }
        }
        if (POOL != 2 && kn && P.qmode) {
            // score(kpos) as the reference sums it (peakcall.cpp:203-209):
            // the hit at kpos - bw + t adds kernel[2bw - t] * countSum, in
            // ascending t; each lane forms its products, the hits' products
            // are compacted in order and added up from LDS broadcasts
            double f = 0.0, r = 0.0;
#pragma unroll
            for (int q = 0; q < kPK; ++q) {
                const int t = 64 * q + lane;
                const bool in = t <= 2 * bw;
                const double kw = ktab[2 * bw - t];  // padded table: in range
                const bool hf = in && nz(pkf[q]);
                const double vf = hf ? kw * (double)pkf[q] : 0.0;
                bool hr = false;
                double vr = 0.0;
                if constexpr (NONDIR) {
                    hr = in && nz(pkr[NONDIR ? q : 0]);
                    vr = hr ? kw * (double)pkr[NONDIR ? q : 0] : 0.0;
                }
                const uint64_t m = __ballot(hf || hr);
                if (hf || hr) {
                    const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    terms[k] = make_double2(vf, vr);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int nh = __builtin_popcountll(m);
                int k = 0;
                for (; k + kTermBatch <= nh; k += kTermBatch) {
                    double2 v[kTermBatch];
#pragma unroll
                    for (int i = 0; i < kTermBatch; ++i) v[i] = terms[k + i];
#pragma unroll
                    for (int i = 0; i < kTermBatch; ++i) {
                        f = f + v[i].x;  // a +0 of the other strand leaves a sum as it is
                        r = r + v[i].y;
                    }
                }
                for (; k < nh; ++k) {
                    const double2 a = terms[k];
                    f = f + a.x;
                    r = r + a.y;
                }
                __builtin_amdgcn_wave_barrier();  // terms reused
            }
            best = NONDIR ? f + r : f;
        }
        if (!kn) {
        if constexpr (POOL == 0) {
            fetch_raw(nf, 0, left);
            if constexpr (NONDIR) fetch_raw(nr, 1, left);
        }
        for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64, ++blk) {
            const int64_t x = x0 + lane;
            const bool valid = x <= (int64_t)right;
            const int nvalid = (int)(((int64_t)right - x0 + 1) < 64 ? ((int64_t)right - x0 + 1) : 64);
            WinT<POOL> cf[NWT];
            uint64_t hf[NWT];
            WinT<POOL> cr[NONDIR ? NWT : 1];
            uint64_t hr[NONDIR ? NWT : 1];
            if constexpr (POOL == 0) {
                const int64_t xb = x0 - 64 * NH;
#pragma unroll
                for (int w = 0; w < NWT; ++w) {
                    cf[w] = nf[w] == kEsc ? ovf_lookup(U, (uint32_t)P.nc[0], (uint32_t)(xb + 64 * w + lane)) : nf[w];
                    if constexpr (NONDIR)
                        cr[w] = nr[w] == kEsc ? ovf_lookup(U, (uint32_t)(S + P.nc[0]), (uint32_t)(xb + 64 * w + lane)) : nr[w];
                }
                if (x0 + 64 <= (int64_t)right) {
                    fetch_raw(nf, 0, x0 + 64);
                    if constexpr (NONDIR) fetch_raw(nr, 1, x0 + 64);
                }
#pragma unroll
                for (int w = 0; w < NWT; ++w) {
                    hf[w] = __ballot(cf[w] != 0u);
                    if constexpr (NONDIR) hr[w] = __ballot(cr[w] != 0u);
                }
            } else {
                region_words<NH, POOL>(cf, hf, U, 0, x0, lane, P);
                if constexpr (NONDIR) region_words<NH, POOL>(cr, hr, U, 1, x0, lane, P);
            }
            double f = kde_word<NWT, NH, NH>(cf, hf, wm, lane, bw, ktab);
            double r = 0.0;
            uint64_t hr_c = 0;
            if constexpr (NONDIR) {
                r = kde_word<NWT, NH, NH>(cr, hr, wm, lane, bw, ktab);
                hr_c = hr[NH];
            }
            const double score = NONDIR ? f + r : f;
            // (K1q runs: the first position joined by a leap with peakPos 0,
            // so Region::addPos re-seeds the peak at the next one, data.cpp:98-101)
            if (valid && (!P.q11 || x > (int64_t)left) && (best_x < 0 || score > best)) {
                best = score;
                best_x = x;
            }
            if (NONDIR && P.want_corr) {
                // pass 3 reads f, r back from this wave's slab instead of
                // recomputing the KDE
                const int64_t off = x0 - (int64_t)left;
                if (cslab && off + 64 <= (int64_t)P.corr_cap) cslab[off + lane] = make_double2(f, r);
                // the two sums stay sequential in position order
                // (data.cpp:22-30): each position's (f, r) is read back as a
                // wave-uniform LDS broadcast (one ds_read_b128 per position
                // instead of four readlanes)
                terms[lane] = make_double2(f, r);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                int l = 0;
                for (; l + kTermBatch <= nvalid; l += kTermBatch) {  // a batch of reads in flight
                    double2 v[kTermBatch];
#pragma unroll
                    for (int i = 0; i < kTermBatch; ++i) v[i] = terms[l + i];
#pragma unroll
                    for (int i = 0; i < kTermBatch; ++i) {
                        sf = sf + v[i].x;
                        sr = sr + v[i].y;
                    }
                }
                for (; l < nvalid; ++l) {
                    const double2 v = terms[l];
                    sf = sf + v.x;
                    sr = sr + v.y;
                }
                __builtin_amdgcn_wave_barrier();  // terms reused by the next word
            }
            // stored hit vectors (peakcall.cpp:210-219; quirk Q7)
            const bool sf_hit = (hf[NH] >> lane) & 1, sr_hit = (hr_c >> lane) & 1;
            uint32_t pc = 0;
            if (POOL == 0 && S == 1) {  // the only sample is the pooled one
                if (valid) {
                    if (sf_hit) pc += (uint32_t)cf[NH];
                    if (NONDIR && sr_hit) pc += (uint32_t)cr[NONDIR ? NH : 0];
                }
                esum1 += pc;
            } else if (kRS) {
                // the pooled non-control count is the word's own centre
                // value; control samples per word (their exptSums count
                // pooled hits only); the non-controls' exptSums come from
                // the plane range sums after the pass (nc_range_sums)
                if (valid) {
                    if (sf_hit) pc += (uint32_t)cf[NH];
                    if (NONDIR && sr_hit) pc += (uint32_t)cr[NONDIR ? NH : 0];
                }
                for (int s = 0; s < S && P.nnc < S; ++s) {
                    if (!P.is_control[s]) continue;
                    uint32_t c = 0;
                    if (valid) {
                        if (sf_hit) c += count_at(U, S, 0, s, x);
                        if (NONDIR && sr_hit) c += count_at(U, S, 1, s, x);
                    }
                    pc += c;
                    const uint32_t t = wave_sum_u32(c);
                    add_es(esum, esl, s, t, lane);
                }
            } else {
                for (int s = 0; s < S; ++s) {
                    uint32_t c = 0;
                    if (valid) {
                        if (sf_hit) c += count_at(U, S, 0, s, x);
                        if (NONDIR && sr_hit) c += count_at(U, S, 1, s, x);
                    }
                    pc += c;
                    const uint32_t t = wave_sum_u32(c);
                    add_es(esum, esl, s, t, lane);
                }
            }
            if (blk < kStatCache) pcache[64 * blk + lane] = pc;
            cnt_acc += pc;
            sum_acc += pc * (uint32_t)(uint16_t)(x - left);
        }
        // peak: first maximum (Region::addPos, data.cpp:98-101)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double ob = __shfl_xor(best, o);
            const long long ox = __shfl_xor((long long)best_x, o);
            if (ox >= 0 && (best_x < 0 || ob > best || (ob == best && ox < best_x))) {
                best = ob;
                best_x = ox;
            }
        }
        }  // !kn
        if (kRS && S > 1 && !staged) nc_range_sums<NONDIR>(esum, esl, U, P, left, right, lane, (uint32_t *)terms);
        if (POOL == 0 && S == 1) {
            const uint32_t t = wave_sum_u32(esum1);
            esum[0] = lane == 0 ? t : 0u;
        }
        const uint32_t count = wave_sum_u32(cnt_acc);
        const uint32_t psum = wave_sum_u32(sum_acc);

        // next region's count bytes (its descriptor arrived during pass 1)
        pre_ok = false;
        if constexpr (kPrefetch) {
            if (known && S == 1 && rn < nreg) {
                const uint32_t ln = rl_u(dsc_n, 0), rgn = rl_u(dsc_n, 1);
                const int nwn = (int)((rgn - ln) / 64u) + 1;
                if (nwn <= kStatCache) {
                    const UnitDesc Un = P.units[rl_u(dsc_n, 2)];
                    gu8 *tn = track_u8(Un, S, 0, P.nc[0]) + fbyte(kPadPos + (int64_t)ln - 1 + lane);
#pragma unroll
                    for (int w = 0; w < kStatCache; ++w) praw[w] = w < nwn ? tn[kWordBytes * w] : 0u;
                    pre_ok = true;
                }
            }
            // and the bytes of its peak's window (Q keys; a run over strip
            // edges finds its peak position later)
            pk_pre = false;
            if (known && P.qmode && rn < nreg && rl_u(dsc_n, 3) != 0) {
                pk_pos = rl_u(dsc_n, 3);
                const UnitDesc Un = P.units[rl_u(dsc_n, 2)];
                const int64_t n0 = kPadPos + (int64_t)pk_pos - bw - 1 + lane;
                gu8 *tp = track_u8(Un, S, 0, P.nc[0]) + fbyte(n0);
#pragma unroll
                for (int w = 0; w < (kPrefetch ? 2 * NH : 1); ++w) pkraw[w] = tp[kWordBytes * w];
                pk_pre = true;
            }
        }
        // ---- pass 2: kurtosis (data.cpp:164-182; powi semantics) ----
        const double x_bar = (double)psum / (double)count;
        double sum2 = 0.0, sum4 = 0.0;
        int blk2 = 0;
        for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64, ++blk2) {
            const int64_t x = x0 + lane;
            const bool valid = x <= (int64_t)right;
            uint32_t pc = 0;
            if (blk2 < kStatCache) {
                pc = pcache[64 * blk2 + lane];
            } else {
                double c0 = 0.0, c1 = 0.0;
                // pooled count at x itself, per strand, to know what was stored
                if (valid) {
                    if (POOL == 0) {
                        c0 = (double)count_at(U, S, 0, P.nc[0], x);
                        if (NONDIR) c1 = (double)count_at(U, S, 1, P.nc[0], x);
                    } else {
                        for (int k = 0; k < P.nnc; ++k) {
                            const double q = POOL == 2 ? P.coef[k] : 1.0;
                            const uint32_t a = count_at(U, S, 0, P.nc[k], x);
                            c0 = POOL == 2 ? c0 + (double)a * q : c0 + (double)a;
                            if (NONDIR) {
                                const uint32_t b = count_at(U, S, 1, P.nc[k], x);
                                c1 = POOL == 2 ? c1 + (double)b * q : c1 + (double)b;
                            }
                        }
                        if (POOL == 2) {
                            for (int k = 0; k < P.nnc; ++k) {
                                c0 = c0 + (double)count_at(U, S, 0, P.nc[k], x);
                                if (NONDIR) c1 = c1 + (double)count_at(U, S, 1, P.nc[k], x);
                            }
                        }
                    }
                }
                const bool h0 = valid && c0 != 0.0, h1 = valid && NONDIR && c1 != 0.0;
                for (int s = 0; s < S; ++s) {
                    if (h0) pc += count_at(U, S, 0, s, x);
                    if (h1) pc += count_at(U, S, 1, s, x);
                }
            }
            // every lane forms its own terms; only the two sums stay
            // sequential, in position order (data.cpp:166-177)
            const double d = (double)(uint16_t)(x - left) - x_bar;
            const double d2 = d * d;
            const double t2 = (double)pc * d2, t4 = (double)pc * (d2 * d2);
            // positions holding a stored hit vector, compacted in position
            // order; the two chains then read them back as wave-uniform LDS
            // broadcasts (one ds_read_b128 per term pair, a batch in flight)
            const uint64_t m = __ballot(pc != 0u);
            const int nh = __builtin_popcountll(m);
            if (pc != 0u) {
                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                terms[k] = make_double2(t2, t4);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int k = 0;
            for (; k + kTermBatch <= nh; k += kTermBatch) {
                double2 v[kTermBatch];
#pragma unroll
                for (int i = 0; i < kTermBatch; ++i) v[i] = terms[k + i];
#pragma unroll
                for (int i = 0; i < kTermBatch; ++i) {
                    sum2 = sum2 + v[i].x;
                    sum4 = sum4 + v[i].y;
                }
            }
            for (; k < nh; ++k) {
                const double2 a = terms[k];
                sum2 = sum2 + a.x;
                sum4 = sum4 + a.y;
            }
            __builtin_amdgcn_wave_barrier();  // terms reused by the next word
        }
        const double kurt = ((double)count - 1) * sum4 / (sum2 * sum2);

        // ---- pass 3: strandCorr(0) (data.cpp:38-58, 184-193) ----
        const uint32_t n = right - left + 1;
        double corr = __builtin_nan("");
        if (NONDIR && P.want_corr && n > 3) {
            const double m1 = sf / (double)n, m2 = sr / (double)n;
            double ss1 = 0.0, ss2 = 0.0, ssr = 0.0;
            const bool cached = cslab && (uint64_t)n + 63 <= P.corr_cap;
            double *prod = (double *)pcache;  // 64 x (p1, p2, p3); pass 2 is done with pcache
            for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64) {
                const int nvalid = (int)(((int64_t)right - x0 + 1) < 64 ? ((int64_t)right - x0 + 1) : 64);
                double f, r;
                if (cached) {
                    const double2 v = cslab[x0 - (int64_t)left + lane];
                    f = v.x;
                    r = v.y;
                } else {
                    WinT<POOL> cf[NWT], cr[NWT];
                    uint64_t hf[NWT], hr[NWT];
                    region_words<NH, POOL>(cf, hf, U, 0, x0, lane, P);
                    region_words<NH, POOL>(cr, hr, U, 1, x0, lane, P);
                    f = kde_word<NWT, NH, NH>(cf, hf, wm, lane, bw, ktab);
                    r = kde_word<NWT, NH, NH>(cr, hr, wm, lane, bw, ktab);
                }
                const double d1 = f - m1, d2 = r - m2;
                prod[3 * lane] = d1 * d1;
                prod[3 * lane + 1] = d2 * d2;
                prod[3 * lane + 2] = d1 * d2;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                int l = 0;
                for (; l + kTermBatch <= nvalid; l += kTermBatch) {  // sequential sums, broadcast reads in flight
                    double v[3 * kTermBatch];
#pragma unroll
                    for (int i = 0; i < 3 * kTermBatch; ++i) v[i] = prod[3 * l + i];
#pragma unroll
                    for (int i = 0; i < kTermBatch; ++i) {
                        ss1 = ss1 + v[3 * i];
                        ss2 = ss2 + v[3 * i + 1];
                        ssr = ssr + v[3 * i + 2];
                    }
                }
                for (; l < nvalid; ++l) {
                    ss1 = ss1 + prod[3 * l];
                    ss2 = ss2 + prod[3 * l + 1];
                    ssr = ssr + prod[3 * l + 2];
                }
                __builtin_amdgcn_wave_barrier();
            }
            const double sd1 = sqrt(ss1 / ((double)n - 1));
            const double sd2 = sqrt(ss2 / ((double)n - 1));
            corr = ssr / (((double)n - 1) * sd1 * sd2);
        }

        // ---- processRegion filters (peakcall.cpp:33-53) ----
        // exptSums: lane s % 64 holds sample s (slot s / 64); one coalesced row
        uint32_t nc_part = 0;
        if (esl) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int s = lane; s < S; s += 64) {
                const uint32_t v = esl[s];
                if (!P.is_control[s]) nc_part += v;
                P.out_counts[ri * S + s] = v;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int s = 64 * q + lane;
                if (s < S) {
                    if (!P.is_control[s]) nc_part += esum[q];
                    P.out_counts[ri * S + s] = esum[q];
                }
            }
        }
        const uint32_t nonctl = wave_sum_u32(nc_part);  // HitCount sum (wraps like the reference)
        bool acc = (double)nonctl >= P.hit_thr;
        if (acc) acc = P.kurt_thr == 0 || (n > 1 && kurt <= P.kurt_thr);
        if (acc) acc = P.corr_thr <= -1 || corr >= P.corr_thr;
        // the 56-byte record as 7 words from lanes 0..6 (one write burst)
        if (lane < 7) {
            uint64_t w;
            switch (lane) {
            case 0: w = (uint64_t)u | ((uint64_t)left << 32); break;
            case 1: w = (uint64_t)right | ((uint64_t)(uint32_t)best_x << 32); break;
            case 2: w = (uint64_t)count | ((uint64_t)nonctl << 32); break;
            case 3: w = (uint64_t)(uint32_t)(acc ? 1 : 0) | ((uint64_t)UP_CLOSE_RULE << 32); break;
            case 4: w = (uint64_t)__double_as_longlong(best); break;
            case 5: w = (uint64_t)__double_as_longlong(kurt); break;
            default: w = (uint64_t)__double_as_longlong(corr); break;
            }
            ((uint64_t *)P.out)[ri * 7 + lane] = w;
        }
        dsc = dsc_n;
    }
}

// ------------------------------------------------------------------------
// K4: strandCorr(shift) for shift = 0..max_shift (src/strand_shift.cpp:
// 205-217, Region::strandCorr, misc/data.cpp:22-58, 184-193).  One block of
// kShiftThreads (three waves) per region, grid-stride over the regions:
//  1. the region's f and r (same KDE as K3) are materialised by the three
//     waves, 64 positions per wave step, into LDS (regions up to
//     kShiftLds positions; longer ones, and replayed regions, which arrive
//     with the scores the state machine stored, use the global slab);
//  2. thread t takes shifts t, t + 192, ...: the reference's sums -- mean of
//     f[0, m), mean of r[2s, 2s + m), the two sums of squared deviations and
//     the cross sum, each sequential in index order -- as three loops whose
//     independent chains (s1 | s2, q1 | q2, q3) interleave, the loads of four
//     iterations issued ahead of their in-order adds.
// ------------------------------------------------------------------------
constexpr int kShiftThreads = 192;
constexpr int kShiftLds = 2048;  // positions of f and r kept in LDS per region
constexpr size_t kShiftLdsBytes = kKTab * sizeof(double) + 2 * kShiftLds * sizeof(double);
// With best != nullptr the table is not written: the block reduces it to
// the reference's choice (strand_shift.cpp:209-217: shifts ascending,
// `corr > bestCorr` from bestCorr = -1, bestShift = 0; NaN never wins), i.e.
// the smallest shift holding the largest correlation above -1.
template <int NH, int POOL>
__global__ void __launch_bounds__(kShiftThreads) shift_kernel(StatParams P, const uint64_t *idx, uint32_t n,
                                                              int max_shift, const uint64_t *slab_off,
                                                              double *slab, const uint8_t *prefilled,
                                                              double *out, uint16_t *best,
                                                              double *best_corr) {
    extern __shared__ double lds_[];
    __shared__ double red_c[kShiftThreads];
    __shared__ int red_s[kShiftThreads];
    const int bw = P.bw;
    const double *ktab = load_ktab(lds_, P.kern, bw);
    double *lf = lds_ + kKTab, *lr = lf + kShiftLds;
    constexpr int NWT = 2 * NH + 1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int nwv = kShiftThreads / 64;
    uint64_t wm[2 * NH + 1];
#pragma unroll
    for (int d = -NH; d <= NH; ++d) wm[d + NH] = win_mask(d, bw);
    for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
        const uint64_t ri = idx[j];
        const uint32_t left = P.starts[ri], right = P.ends[ri], u = P.reg_unit[ri];
        const UnitDesc U = P.units[u];
        const uint32_t len = right - left + 1;
        const bool pre = prefilled[j] != 0;
        const bool in_lds = !pre && len <= (uint32_t)kShiftLds;
        double *fs = in_lds ? lf : slab + slab_off[j];
        double *rs = in_lds ? lr : fs + len;
        // replayed regions arrive with their stored scores; the others are
        // materialised from the dense KDE
        for (int64_t x0 = (int64_t)left + 64 * wv; !pre && x0 <= (int64_t)right; x0 += 64 * nwv) {
            WinT<POOL> cf[NWT], cr[NWT];
            uint64_t hf[NWT], hr[NWT];
            region_words<NH, POOL>(cf, hf, U, 0, x0, lane, P);
            region_words<NH, POOL>(cr, hr, U, 1, x0, lane, P);
            const double f = kde_word<NWT, NH, NH>(cf, hf, wm, lane, bw, ktab);
            const double r = kde_word<NWT, NH, NH>(cr, hr, wm, lane, bw, ktab);
            const int64_t x = x0 + lane;
            if (x <= (int64_t)right) { fs[x - left] = f; rs[x - left] = r; }
        }
        __syncthreads();  // (global slab writes: visible block-wide after the barrier too)
        double bc = -1.0;  // this thread's first maximum over its shifts (ascending)
        int bs = 0;
        for (int sh = threadIdx.x; sh <= max_shift; sh += kShiftThreads) {
            double c = __builtin_nan("");
            if (len > (uint32_t)(2 * sh + 3)) {
                const uint32_t m = len - 2 * sh;
                const double *a = fs, *b = rs + 2 * sh;
                constexpr uint32_t U4 = 4;
                const uint32_t m4 = m & ~(U4 - 1);
                double s1 = 0.0, s2 = 0.0;
                uint32_t i = 0;
                for (; i < m4; i += U4) {
                    double x[U4], y[U4];
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) { x[k] = a[i + k]; y[k] = b[i + k]; }
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) { s1 = s1 + x[k]; s2 = s2 + y[k]; }
                }
                for (; i < m; ++i) { s1 = s1 + a[i]; s2 = s2 + b[i]; }
                const double m1 = s1 / (double)m, m2 = s2 / (double)m;
                double q1 = 0.0, q2 = 0.0;
                for (i = 0; i < m4; i += U4) {
                    double x[U4], y[U4];
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) { x[k] = a[i + k] - m1; y[k] = b[i + k] - m2; }
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) { q1 = q1 + x[k] * x[k]; q2 = q2 + y[k] * y[k]; }
                }
                for (; i < m; ++i) {
                    const double x = a[i] - m1, y = b[i] - m2;
                    q1 = q1 + x * x;
                    q2 = q2 + y * y;
                }
                const double sd1 = sqrt(q1 / ((double)m - 1)), sd2 = sqrt(q2 / ((double)m - 1));
                double q3 = 0.0;
                for (i = 0; i < m4; i += U4) {
                    double x[U4];
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) x[k] = (a[i + k] - m1) * (b[i + k] - m2);
#pragma unroll
                    for (uint32_t k = 0; k < U4; ++k) q3 = q3 + x[k];
                }
                for (; i < m; ++i) q3 = q3 + (a[i] - m1) * (b[i] - m2);
                c = q3 / (((double)m - 1) * sd1 * sd2);
            }
            if (best) {
                if (c > bc) { bc = c; bs = sh; }
            } else {
                out[(uint64_t)j * (max_shift + 1) + sh] = c;
            }
        }
        if (best) {  // larger corr wins, equal corr -> smaller shift
            red_c[threadIdx.x] = bc;
            red_s[threadIdx.x] = bs;
            __syncthreads();
            if (threadIdx.x == 0) {
                double c = -1.0;
                int sbest = 0;
                for (int t = 0; t < kShiftThreads; ++t) {
                    const double v = red_c[t];
                    if (v > c || (v == c && v > -1.0 && red_s[t] < sbest)) { c = v; sbest = red_s[t]; }
                }
                best[j] = (uint16_t)sbest;
                best_corr[j] = c;
            }
        }
        __syncthreads();
    }
}

#ifndef UPK_NH_TU
// ------------------------------------------------------------------------
// aux kernels
// ------------------------------------------------------------------------
// host pairs -> one track (counts >= kEsc become the escape field; the host
// keeps their values in the unit's overflow table).  kPerByte positions share
// a byte, so each pair clears and sets its own field of the dword with
// atomics on disjoint bits (positions within one call are unique).
__global__ void scatter_kernel(uint8_t *track, const uint32_t *__restrict__ pos,
                               const uint32_t *__restrict__ cnt, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t nb = kPadPos + (uint64_t)pos[i] - 1;                  // field index
    uint32_t *word = (uint32_t *)(track + ((uint64_t)fbyte(nb) & ~3ull));  // its aligned dword
    const uint32_t sh = (uint32_t)kTB * (uint32_t)(nb & (4 * kPerByte - 1));
    const uint32_t c = cnt[i] >= kEsc ? kEsc : cnt[i];
    atomicAnd(word, ~(kTMask << sh));
    if (c) atomicOr(word, c << sh);
}

// dense device uint32 counts (position p at src[p-1]) -> one track, one
// dword (4 * kPerByte positions) per thread; counts >= kEsc are appended to
// an overflow list (pos << 32 | count)
__global__ void pack_kernel(uint8_t *track, const uint32_t *__restrict__ src, uint64_t len,
                            unsigned long long *ovf, uint32_t *novf, uint32_t cap) {
    constexpr int PD = 4 * kPerByte;
    const uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * PD;
    if (i0 >= len) return;
    uint32_t out = 0;
#pragma unroll
    for (int k = 0; k < PD; ++k) {
        const uint64_t i = i0 + k;
        uint32_t c = i < len ? src[i] : 0u;
        if (c >= kEsc) {
            const uint32_t slot = atomicAdd(novf, 1u);
            if (slot < cap) ovf[slot] = ((unsigned long long)(i + 1) << 32) | c;
            c = kEsc;
        }
        out |= c << (kTB * k);
    }
    // kPadPos and p-1 = i0 are multiples of PD: one aligned dword store (the
    // fields past len are zero, and the track extends past len + kMaxBw)
    *(uint32_t *)(track + fbyte(kPadPos + (int64_t)i0)) = out;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct SynthThr {
    uint64_t t[6];
};

// synthetic counts are generated into a dense uint32 staging track
// (position p at stage[p-1]) and packed by pack_kernel
// (offset: the track moved by -s positions; what leaves [1, len] is dropped)
__global__ void synth_bg_kernel(uint32_t *stage, uint64_t tkey, int64_t lo, int64_t hi,
                                SynthThr thr, int64_t offset, int64_t len) {
    const int64_t x = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x > hi || x + offset < 1 || x + offset > len) return;
    const uint64_t u = mix64(tkey ^ mix64((uint64_t)x));
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) c += u >= thr.t[k];
    stage[x + offset - 1] = c;
}

// replicate mode's background (peak_seed != 0): the same
// Poisson(λ) per position, drawn sparsely -- chunk c = positions
// [lo + c·2^16, lo + (c+1)·2^16) gets n ~ Poisson(λ·2^16) tags (n = #{k :
// tab[k] <= u0}, tab the 1024 CDF thresholds) at uniform positions (the top 16
// bits of a hash per tag); tags past hi are dropped.  One thread per chunk.
__global__ void synth_bgc_kernel(uint32_t *stage, uint64_t tkey, int64_t lo, int64_t hi,
                                 const uint64_t *__restrict__ tab, int64_t offset, int64_t len,
                                 uint32_t nchunks) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t u0 = mix64(tkey ^ mix64(0x6267000000000000ull + c));
    uint32_t a = 0, b = 1024;
    while (a < b) {
        const uint32_t m = (a + b) >> 1;
        if (tab[m] <= u0) a = m + 1;
        else b = m;
    }
    const int64_t base = lo + ((int64_t)c << 16);
    for (uint32_t i = 0; i < a; ++i) {
        const int64_t x = base + (int64_t)(mix64(u0 ^ mix64((uint64_t)i + 1)) >> 48);
        if (x > hi || x + offset < 1 || x + offset > len) continue;
        atomicAdd(&stage[x + offset - 1], 1u);
    }
}

// the bench's achievable-HBM reference: a float4 (16 B per lane) copy, one
// vector per thread over a grid that covers the buffer (tools/copy_probe.hip
// on MI355X: 6.08 TB/s; grid-stride loops with 1-8 vectors in flight per
// lane, nontemporal or not, and hipMemcpyDtoD reached 4.8-5.55 TB/s)
__global__ void __launch_bounds__(256) hbm_copy_kernel(const u32x4 *__restrict__ a, u32x4 *__restrict__ b,
                                                       uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// sum of a track's counts, escapes excluded (their counts are added on the
// host from the overflow table)
__global__ void track_sum_kernel(const uint8_t *__restrict__ t, uint64_t n, unsigned long long *out) {
    uint64_t acc = 0;
    const u32x4 *v = (const u32x4 *)t;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 x = v[i];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t y = w[k];
            const uint32_t esc = kTB == 4 ? y & (y >> 1) & (y >> 2) & (y >> 3) & 0x11111111u  // fields == 15
                                          : y & (y >> 1) & 0x55555555u;                     // fields == 3
            acc += fsum32(y, 0u) - kEsc * (uint32_t)__builtin_popcount(esc);
        }
    }
    __shared__ unsigned long long red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(out, red[0]);
}

__global__ void synth_peak_kernel(uint32_t *stage, const uint32_t *__restrict__ pos, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&stage[pos[i] - 1], 1u);
}

#endif  // UPK_NH_TU
}  // namespace upk
