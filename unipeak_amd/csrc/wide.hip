// unipeak_amd/csrc/wide.hip -- K1w: the scan for kernels wider than K1's
// register-resident halo (bw > kMaxBw = 511, up to kMaxWideBw = 32,767: a
// window of at most 65,535 cells -- beyond it the reference's UShort
// retirement count wraps, misc/peakcall.cpp:172-177, and the whole-buffer
// replay runs instead; the reference's -b itself is a UShort,
// misc/kernel.hpp:16).  #included by api.hip.
//
// One wave per strip (16,384 positions), directional units with a threshold
// > 0, as K1 (screen + exact) in one kernel:
//  * screen: the strip's window of chunk sums of its screen plane (the one
//    pooled track's plane, or the unit's weighted pooled plane; a saturated
//    255 counts as unbounded) as prefix sums in LDS; a 64-position word can
//    hold a flag only if the weighted tag sum over the union of its
//    positions' windows, [x0 - bw, x0 + 63 + bw], exceeds the budget wskip
//    (the same bound K1a uses);
//  * exact: for each such word every lane sums its position's score over the
//    adds of that window in ascending position -- the order the reference's
//    deque cell receives them (peakcall.cpp:186-209) -- as kern[x - a + bw] *
//    countSum in FP64 (the pooled count words come from load_words, so
//    pooled samples, coefficients and the pooled count track behave as in
//    K1b);
//  * runs, peaks (first maximum) and the strip's record list and edge flags
//    exactly as K1b writes them, so K2 and K3 (known peaks) follow unchanged.
// The tracks of every unit are padded past len + 2bw (unit_stride), so the
// window loads of positions up to len + bw stay in bounds.

namespace upk {

constexpr uint32_t kWideSat = 1u << 18;  // a saturated chunk in the prefix sums
constexpr int kWideChunks = (kStrip + 2 * kMaxWideBw + 64) / 16 + 4;  // 5,127: the widest strip window

template <int POOL>
__global__ void __launch_bounds__(64) wide_kernel(ScanParams P) {
    __shared__ uint32_t pre[kWideChunks + 1];
    const int lane = threadIdx.x;
    const int bw = P.bw;
    const int S = P.S;
    for (uint32_t strip = blockIdx.x; strip < P.nstrips; strip += gridDim.x) {
        const uint32_t u = find_unit(P.units, P.nunits, strip);
        const UnitDesc U = P.units[u];
        const uint32_t local = strip - U.strip0;
        const int64_t p0 = 1 + (int64_t)local * kStrip, pend = p0 + kStrip - 1;
        const int64_t dom_end = (int64_t)U.len + bw;  // the last position a flush retires
        // ---- screen: prefix sums of the window's chunk sums ----
        gu8 *pl = POOL == 0 ? plane_u8(U, S, 0, P.nc[0]) : pooled_u8(U, S);
        const int64_t nchunk_track = (int64_t)(U.stride / 4);
        const int64_t c0 = (kPadPos + (p0 - bw) - 1) >> 4;  // (arithmetic shift: floor)
        const int64_t c1 = (kPadPos + (pend + bw) - 1) >> 4;
        const int nch = (int)(c1 - c0 + 1);
        __syncthreads();  // the previous strip's readers are done
        if (lane == 0) pre[0] = 0u;
        uint32_t carry = 0;
        for (int base = 0; base < nch; base += 64) {
            const int i = base + lane;
            const int64_t c = c0 + i;
            uint32_t v = 0;
            if (i < nch && c >= 0 && c < nchunk_track) {
                v = pl[c];
                v = v == 255u ? kWideSat : v;
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)v, o);
                if (lane >= o) v += y;
            }
            if (i < nch) pre[i + 1] = carry + v;
            carry += (uint32_t)__shfl((int)v, 63);
        }
        __syncthreads();
        // candidate words: lane l decides words l, l + 64, l + 128, l + 192
        uint64_t cand[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t x0 = p0 + 64 * (64 * q + lane);
            const int64_t lo = ((kPadPos + x0 - bw - 1) >> 4) - c0, hi = ((kPadPos + x0 + 63 + bw - 1) >> 4) - c0;
            const uint32_t sum = pre[hi + 1] - pre[lo];
            cand[q] = __ballot(x0 <= dom_end && (sum > P.wskip || sum >= kWideSat));
        }
        // ---- exact scores, runs and records (K1b's record protocol) ----
        RecList R_{0, 0, kInline};
        uint64_t F0 = 0;
        bool open = false, pk_ok = false;
        double best = -__builtin_inf();
        uint32_t bpos = 0;
        auto close_run = [&](uint32_t end_pos) {
            rec_end(R_, end_pos, pk_ok ? bpos : 0u, best, P, strip, lane);
            if (!pk_ok && lane == 0) {  // the run open at p0: its part in this strip
                P.spk[4ull * strip] = (uint64_t)__double_as_longlong(best);
                P.spk[4ull * strip + 1] = bpos;
            }
            open = false;
        };
        for (int g = 0; g < kStripWords; ++g) {
            const int64_t x0 = p0 + 64 * g;
            const bool cw = (cand[g >> 6] >> (g & 63)) & 1;
            if (!cw) {
                if (open) close_run((uint32_t)(x0 - 1));
                continue;
            }
            const int64_t x = x0 + lane;
            double f = 0.0;
            // the adds of [x0 - bw, x0 + 63 + bw] in ascending position
            const int64_t wb0 = ((x0 - bw - 1) >> 6) * 64 + 1;  // 64-aligned word start (position)
            for (int64_t wb = wb0; wb <= x0 + 63 + bw; wb += 64) {
                if (wb + 63 < 1 || wb > (int64_t)U.len) continue;  // no adds outside 1 .. len
                WinT<POOL> cs[1];
                load_words<1, POOL>(cs, U, S, 0, wb, lane, P.nnc, P.nc, P.coef);
                uint64_t m = __ballot(nz(cs[0]) && wb + lane >= 1 && wb + lane <= (int64_t)U.len);
                while (m) {
                    const int k = __builtin_ctzll(m);
                    m &= m - 1;
                    const int64_t a = wb + k;
                    const double cnt = rl_cs(cs[0], k);
                    const int64_t d = x - a;
                    if (d >= -bw && d <= bw) f = f + P.kern[d + bw] * cnt;
                }
            }
            const bool flag = x <= dom_end && f >= P.thr;
            const uint64_t F = __ballot(flag);
            if (g == 0) F0 = F;
            if (open && !(F & 1ull)) close_run((uint32_t)(x0 - 1));
            // no interior start at p0 (K2 joins it to the previous strip's run)
            uint64_t st = F & ~((F << 1) | ((open || g == 0) ? 1ull : 0ull));
            while (st) {
                const int b = __builtin_ctzll(st);
                st &= st - 1;
                rec_start(R_, (uint32_t)(x0 + b), P, strip, lane);
            }
            // each maximal segment of F: its largest score and the first
            // position holding it (Region::addPos keeps the first maximum)
            uint64_t rem = F;
            while (rem) {
                const int a = __builtin_ctzll(rem);
                const uint64_t t = rem >> a;
                const int len = ~t == 0ull ? 64 - a : __builtin_ctzll(~t);
                const uint64_t seg = (len == 64 ? ~0ull : ((1ull << len) - 1ull)) << a;
                rem &= ~seg;
                const bool in = (seg >> lane) & 1ull;
                const double m = wave_max_d(in ? f : -__builtin_inf());
                const uint64_t at = __ballot(in && f == m);
                const uint32_t pp = (uint32_t)(x0 + __builtin_ctzll(at));
                if (!(a == 0 && open)) {  // a new run
                    best = m;
                    bpos = pp;
                    pk_ok = g != 0 || a != 0;  // one at p0 may continue the previous strip
                } else if (m > best) {
                    best = m;
                    bpos = pp;
                }
                open = true;
                if (a + len < 64) close_run((uint32_t)(x0 + a + len - 1));
            }
        }
        if (open && lane == 0) {  // the run open at the strip's last position: its part here
            P.spk[4ull * strip + 2] = (uint64_t)__double_as_longlong(best);
            P.spk[4ull * strip + 3] = bpos;
        }
        const uint64_t info = (uint64_t)R_.ns | ((uint64_t)R_.ne << 16) | ((F0 & 1ull) << 32) |
                              ((uint64_t)open << 33) | ((uint64_t)(local == 0) << 34) |
                              ((uint64_t)(local + 1 == U.nstrips) << 35) | ((uint64_t)(R_.slot != kInline) << 36);
        if (lane == 0) P.strip_info[strip] = info;
    }
}

}  // namespace upk
