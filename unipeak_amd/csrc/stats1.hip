// unipeak_amd/csrc/stats1.hip -- K3 for one pooled directional sample
// (S == 1, no coefficients, one strand per unit: BASELINE configs[1]) with
// the peaks K1b found.  Included by nh_tu.hip after kernels.hip.
//
// Same outputs, bit for bit, as stats_kernel's path for this case
// (processRegion, misc/peakcall.cpp:33-53; Region::exptSums / posMean /
// posKurtosis, misc/data.cpp:104-182; the peak score, peakcall.cpp:203-209),
// organised around what made that path slow (profiles/r05/phases/: of its
// 0.143 ms, 57 us were per-region load latency, 20 us the count pass
// unrolled over 16 words whatever the region's length, 34 us the kurtosis):
//  * a wave takes a run of consecutive regions -- one unit descriptor for
//    most of them -- and the next region's count bytes arrive as 16-byte
//    lane loads (one wave load per region) during the current region;
//  * the bytes are staged in LDS and read back per 64-position word with a
//    per-lane offset fixed for the region (rolled loops over its words);
//  * pass 1 lists the hit positions as (offset, count) pairs in position
//    order, so the kurtosis terms of pass 2 are formed 64 hits per
//    instruction instead of 64 positions; the two sums then run in position
//    order over LDS broadcasts (data.cpp:166-177).
#pragma once

namespace upk {

constexpr int kS1Stage = 64 * 16;                    // staged region bytes: 64 16-byte pieces
constexpr int kS1Words = kS1Stage / kWordBytes - 1;  // region words staged at once (63 at 2 bits)
constexpr int kS1PkStage = 2 * ((kMaxBw + 64) / 64) * kWordBytes + 32;  // the peak window's bytes (2NH words)
constexpr uint32_t kS1Pairs = 320;                   // hit pairs listed per region (more: per-word pass 2)
constexpr int kS1WaveBytes = kS1Stage + kS1PkStage + (int)kS1Pairs * 8 + 64 * 16;
constexpr size_t kStat1Lds = kKTab * sizeof(double) + 4 * (size_t)kS1WaveBytes;
static_assert(kS1Stage % 16 == 0 && kS1PkStage % 16 == 0 && (kS1Pairs * 8) % 16 == 0, "LDS areas 16-byte aligned");

// 16-byte pieces covering the field bytes of positions [first, last] (the
// first byte rounded down to 16): lane l < n loads piece l
struct Span {
    int64_t base;  // first byte (16-aligned)
    int n;         // pieces
};
__device__ __forceinline__ Span span_of(int64_t first_pos, int64_t last_pos) {
    const int64_t b0 = fbyte(kPadPos + first_pos - 1) & ~(int64_t)15;
    const int64_t b1 = fbyte(kPadPos + last_pos - 1);
    return Span{b0, (int)((b1 - b0) / 16 + 1)};
}
__device__ __forceinline__ u32x4 span_load(gu8 *track, const Span &sp, int lane) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (lane < sp.n) v = *((gu32x4 *)(track + sp.base) + lane);
    return v;
}
__device__ __forceinline__ bool piece_esc(const u32x4 &v) {
    return (fbig32(v.x) | fbig32(v.y) | fbig32(v.z) | fbig32(v.w)) != 0u;
}

template <int NH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) stats1_kernel(StatParams P) {
    extern __shared__ double lds_[];
    const int bw = P.bw;
    const double *ktab = load_ktab(lds_, P.kern, bw);
    constexpr int NWT = 2 * NH + 1;
    constexpr int kPK = 2 * NH;  // peak window words (positions kpos - bw .. kpos + bw)
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    uint8_t *wb = (uint8_t *)(lds_ + kKTab) + (threadIdx.x >> 6) * kS1WaveBytes;
    uint8_t *stg = wb;              // the region's count bytes
    uint8_t *pstg = wb + kS1Stage;  // its peak window's bytes
    uint2 *pairs = (uint2 *)(wb + kS1Stage + kS1PkStage);
    double2 *terms = (double2 *)(wb + kS1Stage + kS1PkStage + kS1Pairs * 8);
    const uint64_t nreg = *P.nreg < P.cap ? *P.nreg : P.cap;
    uint64_t wm[NWT];
#pragma unroll
    for (int d = -NH; d <= NH; ++d) wm[d + NH] = win_mask(d, bw);
    const int nc0 = P.nc[0];
    const uint32_t trk = (uint32_t)nc0;  // (strand 0) * S + sample
    const bool ctl0 = P.is_control[0] != 0;

    // a run of consecutive regions per wave
    const uint64_t per = (nreg + nwaves - 1) / nwaves;
    const uint64_t rbeg = (uint64_t)wave * per < nreg ? (uint64_t)wave * per : nreg;
    const uint64_t rend = rbeg + per < nreg ? rbeg + per : nreg;
    auto desc_load = [&](uint64_t r) -> uint32_t {  // lanes 0..5: start, end, unit, peak, peak value
        if (lane >= 6) return 0u;
        const uint32_t *src = lane == 0   ? P.starts + r
                              : lane == 1 ? P.ends + r
                              : lane == 2 ? P.reg_unit + r
                              : lane == 3 ? P.peak_pos + r
                                          : (const uint32_t *)(P.peak_val + r) + (lane - 4);
        return *src;
    };
    uint32_t ucur = 0xFFFFFFFFu;
    UnitDesc U{};
    gu8 *track = nullptr;
    auto track_of = [&](uint32_t u) -> gu8 * {
        if (u == ucur) return track;
        const UnitDesc Un = P.units[u];
        return (gu8 *)Un.base + (uint64_t)nc0 * Un.stride;
    };
    // the terms in terms[0, n) added in order to the two chains (wave-uniform
    // LDS broadcasts, kTermBatch in flight)
    auto chain = [&](int n, double &a, double &b) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int k = 0;
        for (; k + kTermBatch <= n; k += kTermBatch) {
            double2 v[kTermBatch];
#pragma unroll
            for (int i = 0; i < kTermBatch; ++i) v[i] = terms[k + i];
#pragma unroll
            for (int i = 0; i < kTermBatch; ++i) {
                a = a + v[i].x;
                b = b + v[i].y;
            }
        }
        for (; k < n; ++k) {
            const double2 v = terms[k];
            a = a + v.x;
            b = b + v.y;
        }
        __builtin_amdgcn_wave_barrier();  // terms reused
    };
    // compact this lane's term (when h) after the earlier lanes' into terms
    auto compact = [&](bool h, double x, double y) -> int {
        const uint64_t m = __ballot(h);
        if (h) {
            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            terms[k] = make_double2(x, y);
        }
        return __builtin_popcountll(m);
    };

    uint32_t dsc = rbeg < rend ? desc_load(rbeg) : 0u;
    u32x4 pv = {0u, 0u, 0u, 0u}, ppv = {0u, 0u, 0u, 0u};  // the next region's pieces (bytes, peak window)
    bool pv_ok = false, ppv_ok = false;
    for (uint64_t ri = rbeg; ri < rend; ++ri) {
        const uint32_t left = rl_u(dsc, 0), right = rl_u(dsc, 1), u = rl_u(dsc, 2);
        const uint64_t rn = ri + 1;
        const uint32_t dsc_n = rn < rend ? desc_load(rn) : 0u;
        if (u != ucur) {
            U = P.units[u];
            ucur = u;
            track = (gu8 *)U.base + (uint64_t)nc0 * U.stride;
        }
        uint32_t kpos = rl_u(dsc, 3);
        double kval = __longlong_as_double((long long)(((uint64_t)rl_u(dsc, 5) << 32) | rl_u(dsc, 4)));
        const bool pre = kpos != 0;  // the peak window's bytes came with the descriptor's
        if (kpos == 0) {
            // the run crossed a strip edge: first maximum over its parts, in
            // position order (as stats_kernel)
            const uint32_t sa = U.strip0 + (left - 1) / kStrip, sb = U.strip0 + (right - 1) / kStrip;
            for (uint32_t s = sa; s <= sb; ++s) {
                const uint32_t sp0 = 1 + (s - U.strip0) * kStrip;
                const bool prt = (s > sa || left == sp0) && s == sb && right < sp0 + kStrip - 1;
                const uint64_t *e = P.spk + 4ull * s + (prt ? 0 : 2);
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
        // a Q key marked +0.5 (the largest Q at two positions): the first
        // maximum of the FP64 scores decides (the region's KDE below)
        const bool kn = !(P.qmode && kval != __builtin_floor(kval));
        const int nw = (int)((right - left) / 64u) + 1;
        const bool staged = nw <= kS1Words;

        // ---- the region's count bytes, staged in LDS ----
        // lane's field of word w: byte off + kWordBytes * w, bits sh (the
        // same for every word: a word is kWordBytes whole bytes)
        const int64_t n0 = kPadPos + (int64_t)left - 1 + lane;
        const uint32_t sh = fshift(n0);
        bool esc = false;
        int off = 0;
        if (staged) {
            const Span sp = span_of(left, right);
            off = (int)(fbyte(n0) - sp.base);
            const u32x4 v = pv_ok ? pv : span_load(track, sp, lane);
            esc = __ballot(lane < sp.n && piece_esc(v)) != 0;
            __builtin_amdgcn_wave_barrier();  // earlier readers of the stage are done
            if (lane < sp.n) *(u32x4 *)(stg + 16 * lane) = v;
        }
        gu8 *tg = track + fbyte(n0);  // regions too long to stage read their bytes directly
        const uint32_t lim = right - left;  // lane offsets past it hold no stored count
        auto count_word = [&](int w) -> uint32_t {
            const uint32_t o = 64u * (uint32_t)w + (uint32_t)lane;
            if (o > lim) return 0u;
            uint32_t c;
            if (staged) {
                c = ((uint32_t)stg[off + kWordBytes * w] >> sh) & kTMask;
                if (esc && c == kEsc) c = ovf_lookup(U, trk, left + o);
            } else {
                c = ((uint32_t)tg[kWordBytes * w] >> sh) & kTMask;
                if (c == kEsc) c = ovf_lookup(U, trk, left + o);
            }
            return c;
        };
        // the peak window (Q keys): lane t of word q holds position kpos - bw + 64q + t
        bool pesc = false;
        int poff = 0;
        uint32_t psh = 0;
        if (kn && P.qmode) {
            const int64_t pn0 = kPadPos + (int64_t)kpos - bw - 1 + lane;
            const Span psp = span_of((int64_t)kpos - bw, (int64_t)kpos - bw + 64 * kPK - 1);
            poff = (int)(fbyte(pn0) - psp.base);
            psh = fshift(pn0);
            const u32x4 v = (pre && ppv_ok) ? ppv : span_load(track, psp, lane);
            pesc = __ballot(lane < psp.n && piece_esc(v)) != 0;
            if (lane < psp.n) *(u32x4 *)(pstg + 16 * lane) = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- the next region's bytes while this one is worked on ----
        pv_ok = ppv_ok = false;
        if (rn < rend) {
            const uint32_t ln = rl_u(dsc_n, 0), rgn = rl_u(dsc_n, 1), un = rl_u(dsc_n, 2), kp = rl_u(dsc_n, 3);
            gu8 *tn = track_of(un);
            if ((rgn - ln) / 64u + 1 <= (uint32_t)kS1Words) {
                pv = span_load(tn, span_of(ln, rgn), lane);
                pv_ok = true;
            }
            if (P.qmode && kp != 0) {
                ppv = span_load(tn, span_of((int64_t)kp - bw, (int64_t)kp - bw + 64 * kPK - 1), lane);
                ppv_ok = true;
            }
        }

        // ---- pass 1: exptSums, count and position moments; hit pairs ----
        uint32_t bc = 0, bs = 0, np = 0;
        for (int w = 0; w < nw; ++w) {
            const uint32_t c = count_word(w);
            const uint32_t key = (uint32_t)(uint16_t)(64 * w + lane);  // Q8: uint16 offsets
            bc += c;
            bs += c * key;
            const uint64_t m = __ballot(c != 0u);
            if (c != 0u && np <= kS1Pairs) {
                const uint32_t k = np + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (k < kS1Pairs) pairs[k] = make_uint2(key, c);
            }
            np += (uint32_t)__builtin_popcountll(m);
        }
        const uint32_t count = wave_sum_u32(bc);
        const uint32_t psum = wave_sum_u32(bs);
        const uint32_t nonctl = ctl0 ? 0u : count;  // S == 1

        // ---- pass 2: kurtosis (data.cpp:164-182; powi semantics) ----
        const double x_bar = (double)psum / (double)count;
        double sum2 = 0.0, sum4 = 0.0;
        if (np <= kS1Pairs) {  // the terms of 64 hits per step
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint32_t k0 = 0; k0 < np; k0 += 64) {
                const uint32_t k = k0 + (uint32_t)lane;
                if (k < np) {
                    const uint2 pr = pairs[k];
                    const double d = (double)pr.x - x_bar;
                    const double d2 = d * d;
                    terms[lane] = make_double2((double)pr.y * d2, (double)pr.y * (d2 * d2));
                }
                chain((int)(np - k0 < 64u ? np - k0 : 64u), sum2, sum4);
            }
        } else {  // many hits: per word, the positions holding a hit compacted
            for (int w = 0; w < nw; ++w) {
                const uint32_t c = count_word(w);
                const double d = (double)(uint16_t)(64 * w + lane) - x_bar;
                const double d2 = d * d;
                const int n = compact(c != 0u, (double)c * d2, (double)c * (d2 * d2));
                chain(n, sum2, sum4);
            }
        }
        const double kurt = ((double)count - 1) * sum4 / (sum2 * sum2);

        // ---- peak ----
        double best = kval;
        int64_t best_x = kpos;
        if (kn && P.qmode) {
            // score(kpos) as the reference sums it (peakcall.cpp:203-209): the
            // hit at kpos - bw + t adds kernel[2bw - t] * countSum, in ascending t
            double f = 0.0, zero = 0.0;
#pragma unroll
            for (int q = 0; q < kPK; ++q) {
                const int t = 64 * q + lane;
                uint32_t c = 0;
                if (t <= 2 * bw) {
                    c = ((uint32_t)pstg[poff + kWordBytes * q] >> psh) & kTMask;
                    if (pesc && c == kEsc) c = ovf_lookup(U, trk, (uint32_t)((int64_t)kpos - bw + t));
                }
                const double kw = ktab[2 * bw - t];  // padded table: in range
                const int n = compact(c != 0u, kw * (double)c, 0.0);
                chain(n, f, zero);
            }
            best = f;
        } else if (!kn) {
            // tied keys: the region's KDE, first maximum of the FP64 scores
            // (Region::addPos, data.cpp:98-101)
            best = 0.0;
            best_x = -1;
            for (int64_t x0 = left; x0 <= (int64_t)right; x0 += 64) {
                const int64_t x = x0 + lane;
                uint32_t cf[NWT];
                uint64_t hf[NWT];
                load_words<NWT, 0>(cf, U, 1, 0, x0 - 64 * NH, lane, 1, P.nc, nullptr);
#pragma unroll
                for (int w = 0; w < NWT; ++w) hf[w] = __ballot(cf[w] != 0u);
                const double f = kde_word<NWT, NH, NH>(cf, hf, wm, lane, bw, ktab);
                if (x <= (int64_t)right && (best_x < 0 || f > best)) {
                    best = f;
                    best_x = x;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(best, o);
                const long long ox = __shfl_xor((long long)best_x, o);
                if (ox >= 0 && (best_x < 0 || ob > best || (ob == best && ox < best_x))) {
                    best = ob;
                    best_x = ox;
                }
            }
        }

        // ---- processRegion filters (peakcall.cpp:33-53); strandCorr is NaN ----
        const uint32_t n = right - left + 1;
        bool acc = (double)nonctl >= P.hit_thr;
        if (acc) acc = P.kurt_thr == 0 || (n > 1 && kurt <= P.kurt_thr);
        if (acc) acc = P.corr_thr <= -1;
        if (lane == 0) P.out_counts[ri] = count;  // exptSums[0]
        if (lane < 7) {  // the 56-byte record as 7 words (one write burst)
            uint64_t w;
            switch (lane) {
            case 0: w = (uint64_t)u | ((uint64_t)left << 32); break;
            case 1: w = (uint64_t)right | ((uint64_t)(uint32_t)best_x << 32); break;
            case 2: w = (uint64_t)count | ((uint64_t)nonctl << 32); break;
            case 3: w = (uint64_t)(uint32_t)(acc ? 1 : 0) | ((uint64_t)UP_CLOSE_RULE << 32); break;
            case 4: w = (uint64_t)__double_as_longlong(best); break;
            case 5: w = (uint64_t)__double_as_longlong(kurt); break;
            default: w = (uint64_t)__double_as_longlong(__builtin_nan("")); break;
            }
            ((uint64_t *)P.out)[ri * 7 + lane] = w;
        }
        dsc = dsc_n;
    }
}

}  // namespace upk

namespace upk {

// ------------------------------------------------------------------------
// K3L: the same statistics with ONE LANE PER REGION (round 6).  A region of
// configs[1] holds ~245 positions and ~107 tags: stats1_kernel's wave spent
// ~15 us per region in dependent loads and wave-wide bookkeeping, 8 regions
// in turn per wave, on every pass's chain stream.  Here each lane stages its
// own region's 2-bit dwords in an LDS row (all loads in flight) and:
//  * pass 1 (exptSums, count, position moments with the Q8 uint16 offsets)
//    per dword from popcounts, escaped fields resolved four dwords at a time
//    from 16-byte escape-tile loads and cached for pass 2;
//  * pass 2 (the two kurtosis sums in position order, data.cpp:164-182,
//    powi semantics) four hits per step: terms formed independently, added
//    in order;
//  * the peak score (the reference's ordered sum over the peak's window,
//    peakcall.cpp:203-209) per staged dword, 16 terms at once (an empty
//    field adds +0.0, exact on the non-negative sum);
// so every FP64 sum has the same operations in the same order as
// stats1_kernel's.  Regions whose Q-key peak is tied (+0.5) get the wave's
// KDE afterwards, one at a time, as do regions above P.heavy hits for pass 2.
// Records are staged in LDS and written as contiguous wave stores.
// Measurements and the variants tried: DESIGN.md §4 "Round 6",
// profiles/r06/ab_k3_walks.txt.
constexpr int kK3LRecWords = 7;  // 56-byte up_region as uint64 words
constexpr int kK3LRow = 32;      // region dwords staged per lane at a time (512 positions)
constexpr int kK3LEsc = 64;      // escaped counts cached per lane (bytes)
constexpr int kK3LRowStride = kK3LRow + 1;  // (odd: the lanes' k-th words fall in distinct banks)
constexpr int kK3LThreads = 128; // two waves per block (the per-lane LDS rows)
constexpr size_t kStat1LLds = kKTab * sizeof(double) + (kK3LThreads / 64) * 64 * kK3LRecWords * sizeof(uint64_t) +
                              kK3LThreads * (kK3LRowStride * sizeof(uint32_t) + kK3LEsc);

template <int NH>
__global__ void __launch_bounds__(kK3LThreads) stats1L_kernel(StatParams P) {
    extern __shared__ double lds_[];
    const int bw = P.bw;
    const double *ktab = load_ktab(lds_, P.kern, bw);
    uint64_t *rstage = (uint64_t *)(lds_ + kKTab) + (threadIdx.x >> 6) * 64 * kK3LRecWords;
    // this lane's staged region dwords and escaped counts
    uint32_t *row = (uint32_t *)((uint64_t *)(lds_ + kKTab) + (kK3LThreads / 64) * 64 * kK3LRecWords) +
                    threadIdx.x * kK3LRowStride;
    uint8_t *ecache = (uint8_t *)((uint32_t *)((uint64_t *)(lds_ + kKTab) + (kK3LThreads / 64) * 64 * kK3LRecWords) +
                                  kK3LThreads * kK3LRowStride) +
                      threadIdx.x * kK3LEsc;
    constexpr int NWT = 2 * NH + 1;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const uint64_t nreg = *P.nreg < P.cap ? *P.nreg : P.cap;
    uint64_t wm[NWT];
#pragma unroll
    for (int d = -NH; d <= NH; ++d) wm[d + NH] = win_mask(d, bw);
    const int nc0 = P.nc[0];
    const uint32_t trk = (uint32_t)nc0;
    const bool ctl0 = P.is_control[0] != 0;

    for (uint64_t base = (uint64_t)wave * 64; base < nreg; base += (uint64_t)nwaves * 64) {
        const uint64_t ri = base + (uint64_t)lane;
        const bool live = ri < nreg;
        const uint64_t rq = live ? ri : base;  // (lanes past the end shadow the wave's first region)
        const uint32_t left = P.starts[rq], right = P.ends[rq], u = P.reg_unit[rq];
        uint32_t kpos = P.peak_pos[rq];
        double kval = P.peak_val[rq];
        const UnitDesc U = P.units[u];
        gu32 *tw = (gu32 *)((gu8 *)U.base + (uint64_t)nc0 * U.stride);
        if (kpos == 0) {  // the run crossed a strip edge: its parts, in position order
            const uint32_t sa = U.strip0 + (left - 1) / kStrip, sb = U.strip0 + (right - 1) / kStrip;
            for (uint32_t s = sa; s <= sb; ++s) {
                const uint32_t sp0 = 1 + (s - U.strip0) * kStrip;
                const bool prt = (s > sa || left == sp0) && s == sb && right < sp0 + kStrip - 1;
                const uint64_t *e = P.spk + 4ull * s + (prt ? 0 : 2);
                const double v = __longlong_as_double((long long)e[0]);
                if (P.qmode) {
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
        const bool kn = !(P.qmode && kval != __builtin_floor(kval));
        if (P.cut == 1) continue;  // (measurement aid: descriptors only)
        // fields of dword j restricted to positions [left, right]
        const int64_t n0 = kPadPos + (int64_t)left - 1, n1 = kPadPos + (int64_t)right - 1;
        const int64_t j0 = n0 >> 4, j1 = n1 >> 4;
        auto dword_at = [&](int64_t j) -> uint32_t {
            uint32_t d = tw[j];
            if (j == j0) d &= ~0u << (2 * (n0 & 15));
            if (j == j1 && (n1 & 15) != 15) d &= (1u << (2 * ((n1 & 15) + 1))) - 1u;
            return d;
        };
        // dwords c0 .. min(c0 + kK3LRow - 1, c1) of the fields [f0, f1] into
        // the lane's row; returns the mask of the nonzero ones.  Every load
        // is unconditional (indices clamped) and lands in registers before
        // the row is written: loads guarded one by one and stored at once
        // compiled to one wait per dword (the first K3L measured 0.22 ms)
        auto stage = [&](int64_t c0, int64_t c1, int64_t f0, int64_t f1) -> uint32_t {
            uint32_t v[kK3LRow];
#pragma unroll
            for (int k = 0; k < kK3LRow; ++k) v[k] = tw[c0 + k <= c1 ? c0 + k : c1];
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < kK3LRow; ++k) {
                const int64_t j = c0 + k;
                uint32_t d = j <= c1 ? v[k] : 0u;
                if (j == (f0 >> 4)) d &= ~0u << (2 * (f0 & 15));
                if (j == (f1 >> 4) && (f1 & 15) != 15) d &= (1u << (2 * ((f1 & 15) + 1))) - 1u;
                row[k] = d;
                m |= (d != 0u ? 1u : 0u) << k;
            }
            return m;
        };
        // every hit (position, count) of the region in ascending position.
        // Regions of up to kK3LRow dwords are staged in the lane's LDS row
        // (every load in flight at once) with a mask of the nonzero dwords,
        // and walked hit by hit -- one field per iteration whatever dword it
        // sits in, so the wave's iterations are its largest region's hits,
        // not the sum over dword slots of every lane's largest dword (a
        // first version with one loop per dword measured 0.22 ms alone).
        // The walks' k-th escaped field is the same field: the first walk
        // caches the counts (kK3LEsc per lane) for the second.
        const int nd = (int)(j1 - j0 + 1);
        const bool staged = nd <= kK3LRow;
        const uint32_t nzm = (live && staged) ? stage(j0, j1, n0, n1) : 0u;
        auto walk = [&](bool cache, auto &&visit) {
            uint32_t ne = 0;  // escaped fields so far
            auto one = [&](uint32_t &d, int64_t j) {
                const int b = __builtin_ctz(d) & ~1;  // the field's low bit
                uint32_t c = (d >> b) & 3u;
                d &= ~(3u << b);
                const int64_t pos = 16 * j + b / 2 - kPadPos + 1;
                if (c == kEsc) {
                    if (cache && ne < (uint32_t)kK3LEsc && ecache[ne] != 255u) {
                        c = ecache[ne];
                    } else {
                        c = ovf_lookup(U, trk, (uint32_t)pos);
                        if (!cache && ne < (uint32_t)kK3LEsc) ecache[ne] = (uint8_t)(c < 255u ? c : 255u);
                    }
                    ++ne;
                }
                visit((uint32_t)pos, c);
            };
            // the hits of the staged chunk starting at dword c0 (mask m)
            auto hits = [&](uint32_t m, int64_t c0) {
                uint32_t d = 0;
                int k = 0;
                for (;;) {
                    if (d == 0u) {
                        if (m == 0u) break;
                        k = __builtin_ctz(m);
                        m &= m - 1u;
                        d = row[k];
                    }
                    one(d, c0 + k);
                }
            };
            if (staged) {
                hits(nzm, j0);
            } else {
                // longer regions: kK3LRow dwords at a time, each chunk's
                // loads in flight together (one dependent load per dword
                // made the longest region of any wave the kernel's time)
                for (int64_t c0 = j0; c0 <= j1; c0 += kK3LRow) hits(stage(c0, j1, n0, n1), c0);
            }
        };
        if (P.cut == 2) continue;  // (+ staging)
        constexpr uint32_t kLo = 0x55555555u;
        // the escape tiles of the region's first two overflow blocks (a
        // staged region spans at most two; longer ones may look up more)
        const uint32_t nblk = ovf_nblk(U.len), b0 = (left - 1u) >> kOvfBlkShift;
        const bool has_ovf = U.ovf != 0;
        uint32_t ti0 = kNoTile, ti1 = kNoTile;
        if (live && has_ovf) {
            gu32 *tix = (gu32 *)U.ovf_tidx + (size_t)trk * nblk;
            ti0 = tix[b0];
            ti1 = tix[b0 + 1u < nblk ? b0 + 1u : b0];
        }
        uint32_t count = 0, psum = 0, nh = 0;  // nh: hits (the second walk's iterations)
        if (live && right - left < 65536u) {
            // no offset wraps (Q8): each dword's count and position moment
            // from popcounts -- sum_f v_f and sum_f f * v_f over its 16
            // fields, the field index's bit q selected by kFb[q] -- so this
            // pass costs dwords, not hits (uint32 arithmetic: exact mod 2^32
            // like the reference's).  Escaped fields hold 3: the true count
            // replaces it, and is cached for the second walk.
            constexpr uint32_t kFb[4] = {0x44444444u, 0x50505050u, 0x55005500u, 0x55550000u};
            uint32_t ne = 0;
            auto moments = [&](uint32_t m, int64_t c0) {
                uint32_t em = 0;  // dwords holding an escaped field
                while (m) {
                    const int k = __builtin_ctz(m);
                    m &= m - 1u;
                    const uint32_t d = row[k];
                    const uint32_t off = (uint32_t)(16 * (c0 + k) - kPadPos + 1) - left;  // field 0's offset
                    const uint32_t s = __builtin_popcount(d & kLo) + 2u * __builtin_popcount(d & ~kLo);
                    uint32_t w = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        w += (__builtin_popcount(d & kFb[q]) + 2u * __builtin_popcount(d & (kFb[q] << 1))) << q;
                    count += s;
                    psum += s * off + w;
                    nh += __builtin_popcount((d | (d >> 1)) & kLo);
                    em |= ((d & (d >> 1) & kLo) != 0u ? 1u : 0u) << k;
                }
                // escaped fields, in position order: a dword's 16 tile bytes
                // (counts up to 254) come as one 16-byte load, four dwords'
                // loads in flight together (one dependent lookup per escape
                // was most of this kernel's time: ~100 tags per region at 2
                // bits leave several escapes in each)
                while (em) {
                    int ks[4];
                    bool ok[4];
                    gu8 *src[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        ok[i] = em != 0u;
                        ks[i] = ok[i] ? __builtin_ctz(em) : ks[0];
                        em &= em - 1u;
                        const uint32_t p1 = (uint32_t)(16 * (c0 + ks[i]) - kPadPos);  // field 0's position - 1
                        const uint32_t blk = p1 >> kOvfBlkShift;
                        const uint32_t ti = blk == b0 ? ti0 : blk == b0 + 1u ? ti1 : kNoTile;
                        src[i] = ti != kNoTile ? (gu8 *)U.ovf_tiles + (size_t)ti * kOvfBlk + (p1 & (kOvfBlk - 1u))
                                               : (gu8 *)P.kern;  // (a safe address; not read)
                    }
                    u32x4 tv[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) tv[i] = *(gu32x4 *)src[i];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (!ok[i]) continue;
                        const uint32_t d = row[ks[i]];
                        const uint32_t off = (uint32_t)(16 * (c0 + ks[i]) - kPadPos + 1) - left;
                        const bool direct = src[i] != (gu8 *)P.kern;
                        for (uint32_t e = d & (d >> 1) & kLo; e; e &= e - 1u) {
                            const uint32_t f = (uint32_t)__builtin_ctz(e) >> 1;
                            const uint32_t q = f >> 2;
                            const uint32_t word = q == 0 ? tv[i].x : q == 1 ? tv[i].y : q == 2 ? tv[i].z : tv[i].w;
                            uint32_t c = (word >> (8 * (f & 3u))) & 255u;
                            if (!has_ovf) {
                                c = kEsc;
                            } else if (!direct || c == 255u) {
                                c = ovf_lookup(U, trk, off + f + left);
                            }
                            if (ne < (uint32_t)kK3LEsc) ecache[ne] = (uint8_t)(c < 255u ? c : 255u);
                            ++ne;
                            count += c - kEsc;
                            psum += (c - kEsc) * (off + f);
                        }
                    }
                }
            };
            if (staged) {
                moments(nzm, j0);
            } else {
                for (int64_t c0 = j0; c0 <= j1; c0 += kK3LRow) moments(stage(c0, j1, n0, n1), c0);
            }
        } else if (live) {
            walk(false, [&](uint32_t pos, uint32_t c) {
                count += c;
                psum += c * (uint32_t)(uint16_t)(pos - left);  // Q8: uint16 offsets
            });
            nh = ~0u;
        }
        const double x_bar = (double)psum / (double)count;
        if (P.cut == 6 && count == 12345u) P.out_counts[0] = (uint32_t)x_bar;  // (+ the first walk)
        if (P.cut == 6) continue;
        double sum2 = 0.0, sum4 = 0.0;
        const bool heavy = live && nh > (uint32_t)P.heavy;
        if (live && !heavy) {
            // per nonzero dword, all 16 fields at once: an empty field's
            // terms are +0.0, which leaves the (non-negative) sums unchanged
            // exactly, so the adds stay the hits' adds in position order
            // while the terms' FP64 work is independent across fields (a
            // loop over hits ran one dependent chain per hit)
            uint32_t ne = 0;
            auto terms = [&](uint32_t m, int64_t c0) {
                while (m) {
                    const int k = __builtin_ctz(m);
                    m &= m - 1u;
                    const uint32_t d = row[k];
                    const uint32_t off = (uint32_t)(16 * (c0 + k) - kPadPos + 1) - left;  // field 0's offset
                    double t2[16], t4[16];
#pragma unroll
                    for (int f = 0; f < 16; ++f) {
                        uint32_t c = (d >> (2 * f)) & 3u;
                        if (c == kEsc) {
                            c = ne < (uint32_t)kK3LEsc && ecache[ne] != 255u ? ecache[ne]
                                                                             : ovf_lookup(U, trk, off + (uint32_t)f + left);
                            ++ne;
                        }
                        const double dd = (double)(uint16_t)(off + (uint32_t)f) - x_bar;
                        const double d2 = dd * dd;
                        t2[f] = c != 0u ? (double)c * d2 : 0.0;
                        t4[f] = c != 0u ? (double)c * (d2 * d2) : 0.0;
                    }
#pragma unroll
                    for (int f = 0; f < 16; ++f) {
                        sum2 = sum2 + t2[f];
                        sum4 = sum4 + t4[f];
                    }
                }
            };
            // or four hits per step: the four found one after another (integer
            // work), their terms formed independently, then added in order --
            // a dword holds ~5 hits, so this forms ~8 terms where the dword
            // form forms 16
            auto hits4 = [&](uint32_t m, int64_t c0) {
                uint32_t d = 0;
                int64_t j = 0;
                for (;;) {
                    uint32_t cv[4], ov[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (d == 0u && m != 0u) {
                            const int k = __builtin_ctz(m);
                            m &= m - 1u;
                            d = row[k];
                            j = c0 + k;
                        }
                        cv[i] = 0u;
                        ov[i] = 0u;
                        if (d != 0u) {
                            const int b = __builtin_ctz(d) & ~1;
                            cv[i] = (d >> b) & 3u;
                            d &= ~(3u << b);
                            ov[i] = (uint32_t)(16 * j + b / 2 - kPadPos + 1) - left;  // pos - left
                        }
                    }
                    if (cv[0] == 0u) break;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (cv[i] == kEsc) {
                            cv[i] = ne < (uint32_t)kK3LEsc && ecache[ne] != 255u ? ecache[ne]
                                                                                 : ovf_lookup(U, trk, ov[i] + left);
                            ++ne;
                        }
                    }
                    double t2[4], t4[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const double dd = (double)(uint16_t)ov[i] - x_bar;
                        const double d2 = dd * dd;
                        t2[i] = cv[i] != 0u ? (double)cv[i] * d2 : 0.0;
                        t4[i] = cv[i] != 0u ? (double)cv[i] * (d2 * d2) : 0.0;
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        sum2 = sum2 + t2[i];
                        sum4 = sum4 + t4[i];
                    }
                }
            };
            if (P.w2hits) {
                if (staged) {
                    hits4(nzm, j0);
                } else {
                    for (int64_t c0 = j0; c0 <= j1; c0 += kK3LRow) hits4(stage(c0, j1, n0, n1), c0);
                }
            } else if (staged) {
                terms(nzm, j0);
            } else {
                for (int64_t c0 = j0; c0 <= j1; c0 += kK3LRow) terms(stage(c0, j1, n0, n1), c0);
            }
        }
        // Regions with many hits would hold the whole wave in their lane's
        // walk: the wave sums their terms instead, one region at a time, 64
        // positions per step -- each step's terms formed by the lanes,
        // compacted in LDS, then added in position order (the same FP64
        // operations in the same order as the lane's walk).  Their dwords
        // come from the lane's staged row, or 64 at a time from HBM.
        uint64_t hv = __ballot(heavy);
        if (hv) {
            double *tx = (double *)rstage, *ty = tx + 64;  // (rstage is free until the records)
            const uint32_t *rows0 = row - threadIdx.x * kK3LRowStride;
            while (hv) {
                const int l = __builtin_ctzll(hv);
                hv &= hv - 1;
                const uint32_t hl = rl_u(left, l), hr = rl_u(right, l), hu = rl_u(u, l);
                const double hx = __shfl(x_bar, l);
                const UnitDesc Uh = P.units[hu];
                gu32 *htw = (gu32 *)((gu8 *)Uh.base + (uint64_t)nc0 * Uh.stride);
                const int64_t hn0 = kPadPos + (int64_t)hl - 1, hn1 = kPadPos + (int64_t)hr - 1;
                const int64_t hj0 = hn0 >> 4, hj1 = hn1 >> 4;
                const bool hst = hj1 - hj0 + 1 <= kK3LRow;  // staged in lane l's row before the walks
                const uint32_t *hrow = rows0 + ((threadIdx.x & ~63u) + (uint32_t)l) * kK3LRowStride;
                double a = 0.0, b = 0.0;
                for (int64_t cb = hj0; cb <= hj1; cb += 64) {
                    uint32_t dv = 0u;
                    if (cb + lane <= hj1) dv = hst ? hrow[lane] : htw[cb + lane];
                    for (int w = 0; w < 16; ++w) {
                        const int64_t g = 16 * cb + 64 * w + lane;  // the lane's field
                        if (16 * cb + 64 * w > hn1) break;
                        const uint32_t d = (uint32_t)__shfl((int)dv, 4 * w + (lane >> 4));
                        uint32_t c = g >= hn0 && g <= hn1 ? (d >> (2 * (lane & 15))) & kTMask : 0u;
                        const int64_t pos = g - kPadPos + 1;
                        if (c == kEsc) c = ovf_lookup(Uh, trk, (uint32_t)pos);
                        const double dd = (double)(uint16_t)(pos - (int64_t)hl) - hx;
                        const double d2 = dd * dd;
                        const uint64_t m = __ballot(c != 0u);
                        if (c != 0u) {
                            const uint32_t k =
                                __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                            tx[k] = (double)c * d2;
                            ty[k] = (double)c * (d2 * d2);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        const int n = __builtin_popcountll(m);
                        for (int k = 0; k < n; ++k) {
                            a = a + tx[k];
                            b = b + ty[k];
                        }
                        __builtin_amdgcn_wave_barrier();  // the terms are reused
                    }
                }
                if (lane == l) {
                    sum2 = a;
                    sum4 = b;
                }
            }
        }
        const double kurt = ((double)count - 1) * sum4 / (sum2 * sum2);
        if (P.cut == 3 && count == 12345u) P.out_counts[0] = (uint32_t)kurt;  // (+ both walks; keep them live)
        if (P.cut == 3) continue;
        double best = kval;
        int64_t best_x = kpos;
        if (live && kn && P.qmode) {
            // score(kpos): the hit at kpos - bw + t adds kernel[2bw - t] *
            // countSum, in ascending t (positions outside the contig read 0)
            const int64_t p0 = (int64_t)kpos - bw, p1 = (int64_t)kpos + bw;
            const int64_t a0 = kPadPos + p0 - 1, a1 = kPadPos + p1 - 1;
            double f = 0.0;
            // the window's dwords staged like the region's (the row is free
            // now), then per nonzero dword all 16 fields' terms at once (an
            // empty field's is +0.0, exact on the non-negative sum) and
            // their adds in position order; a dword's escaped counts come
            // from one 16-byte escape-tile load
            const int64_t q0 = a0 >> 4, q1 = a1 >> 4;
            for (int64_t c0 = q0; c0 <= q1; c0 += kK3LRow) {
                uint32_t m = stage(c0, q1, a0, a1);
                while (m) {
                    const int k = __builtin_ctz(m);
                    m &= m - 1u;
                    const uint32_t d = row[k];
                    const int64_t g0 = 16 * (c0 + k);  // field 0
                    u32x4 tv = {0u, 0u, 0u, 0u};
                    bool direct = false;
                    if ((d & (d >> 1) & kLo) != 0u && has_ovf) {
                        const uint32_t p1f = (uint32_t)(g0 - kPadPos);  // field 0's position - 1 (escapes lie in the contig)
                        const uint32_t blk = p1f >> kOvfBlkShift;
                        const uint32_t ti = blk == b0 ? ti0 : blk == b0 + 1u ? ti1 : kNoTile;
                        if (ti != kNoTile) {
                            tv = *(gu32x4 *)((gu8 *)U.ovf_tiles + (size_t)ti * kOvfBlk + (p1f & (kOvfBlk - 1u)));
                            direct = true;
                        }
                    }
                    double t[16];
#pragma unroll
                    for (int fi = 0; fi < 16; ++fi) {
                        uint32_t c = (d >> (2 * fi)) & 3u;
                        const int64_t g = g0 + fi;
                        if (c == kEsc) {
                            const uint32_t q = (uint32_t)fi >> 2;
                            const uint32_t w = q == 0 ? tv.x : q == 1 ? tv.y : q == 2 ? tv.z : tv.w;
                            const uint32_t v = (w >> (8 * (fi & 3))) & 255u;
                            c = !has_ovf ? kEsc : (direct && v != 255u) ? v : ovf_lookup(U, trk, (uint32_t)(g - kPadPos + 1));
                        }
                        t[fi] = c != 0u ? ktab[2 * bw - (int)(g - a0)] * (double)c : 0.0;
                    }
#pragma unroll
                    for (int fi = 0; fi < 16; ++fi) f = f + t[fi];
                }
            }
            best = f;
        }
        if (P.cut == 4 && count == 12345u) P.out_counts[0] = (uint32_t)best;  // (+ the peak's window)
        if (P.cut == 4) continue;
        // tied Q keys: the region's KDE, first maximum of the FP64 scores
        // (Region::addPos, data.cpp:98-101) -- the wave, one region at a time
        uint64_t tied = __ballot(live && !kn);
        while (tied) {
            const int l = __builtin_ctzll(tied);
            tied &= tied - 1;
            const uint32_t tl = rl_u(left, l), tr = rl_u(right, l), tu = rl_u(u, l);
            const UnitDesc Ut = P.units[tu];
            double tb = 0.0;
            int64_t tx = -1;
            for (int64_t x0 = tl; x0 <= (int64_t)tr; x0 += 64) {
                const int64_t x = x0 + lane;
                uint32_t cf[NWT];
                uint64_t hf[NWT];
                load_words<NWT, 0>(cf, Ut, 1, 0, x0 - 64 * NH, lane, 1, P.nc, nullptr);
#pragma unroll
                for (int w = 0; w < NWT; ++w) hf[w] = __ballot(cf[w] != 0u);
                const double f = kde_word<NWT, NH, NH>(cf, hf, wm, lane, bw, ktab);
                if (x <= (int64_t)tr && (tx < 0 || f > tb)) {
                    tb = f;
                    tx = x;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const double ob = __shfl_xor(tb, o);
                const long long ox = __shfl_xor((long long)tx, o);
                if (ox >= 0 && (tx < 0 || ob > tb || (ob == tb && ox < tx))) {
                    tb = ob;
                    tx = ox;
                }
            }
            if (lane == l) {
                best = tb;
                best_x = tx;
            }
        }
        if (P.cut == 5) continue;  // (+ the tied regions' KDE)
        // processRegion filters (peakcall.cpp:33-53); strandCorr is NaN
        const uint32_t nonctl = ctl0 ? 0u : count;  // S == 1
        const uint32_t n = right - left + 1;
        bool acc = (double)nonctl >= P.hit_thr;
        if (acc) acc = P.kurt_thr == 0 || (n > 1 && kurt <= P.kurt_thr);
        if (acc) acc = P.corr_thr <= -1;
        if (live) {
            P.out_counts[ri] = count;  // exptSums[0]
            uint64_t *r = rstage + (uint64_t)lane * kK3LRecWords;
            r[0] = (uint64_t)u | ((uint64_t)left << 32);
            r[1] = (uint64_t)right | ((uint64_t)(uint32_t)best_x << 32);
            r[2] = (uint64_t)count | ((uint64_t)nonctl << 32);
            r[3] = (uint64_t)(uint32_t)(acc ? 1 : 0) | ((uint64_t)UP_CLOSE_RULE << 32);
            r[4] = (uint64_t)__double_as_longlong(best);
            r[5] = (uint64_t)__double_as_longlong(kurt);
            r[6] = (uint64_t)__double_as_longlong(__builtin_nan(""));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the wave's records as one contiguous area: 8-byte lane stores, 512
        // bytes per instruction (a caller's record target is 8-byte aligned)
        const uint32_t nw = (uint32_t)((nreg - base < 64 ? nreg - base : 64) * kK3LRecWords);
        uint64_t *dst = (uint64_t *)P.out + base * kK3LRecWords;
        for (uint32_t q = (uint32_t)lane; q < nw; q += 64) dst[q] = rstage[q];
        __builtin_amdgcn_wave_barrier();  // rstage reused
    }
}

}  // namespace upk
