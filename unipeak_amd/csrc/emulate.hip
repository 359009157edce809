// unipeak_amd/csrc/emulate.hip -- K0: exact replay of the ProfileBuffer
// state machine (misc/peakcall.cpp:33-231, Region stats misc/data.cpp:92-193)
// for the units the parallel scan cannot represent: a contig pass whose
// pooled hits include a position <= bw (quirk Q1: the deque window does not
// shift there, peakcall.cpp:177-183, and leftover density / an open region
// can leak into the buffer's next contig pass, peakcall.cpp:164-168,
// 224-231).  #included by api.hip.
//
// One workgroup (one wave) per ProfileBuffer walks that buffer's units in
// order.  A chain starts at a unit with a head hit and replays add() for
// every position with tags on the buffer's strand(s) (control samples
// included: control-only adds move the window too).  It stops as soon as the
// replayed state is the one the parallel path assumes -- the buffer is
// aligned (an add past bw happened in this unit), every position that could
// hold misaligned leftovers (<= first aligned add + bw) has been retired and
// no region is open -- and records the resync position X: regions of that
// unit starting at or after X come from K1-K3 unchanged, earlier ones from
// here.  A chain that ends a unit dirty continues into the buffer's next unit.
// The wave runs the state machine in lockstep (identical state in every
// lane): the window update of an add, the per-sample work and a region's
// statistics are split over the lanes, every FP64 sum keeps the reference's
// order (per-lane terms staged in LDS, added up in position order), and the
// wave scans for adds 64 positions at a time.

namespace upk {

struct EmuParams {
    const UnitDesc *units;
    uint32_t nunits;
    const int32_t *unit_buffer;
    // chain groups: group g = units gunits[goff[g] .. goff[g + 1]) of one
    // buffer in its order; groups are independent (each starts from a fresh
    // buffer state), so workgroups take them in parallel (scratch per
    // workgroup slot)
    const uint32_t *gunits, *goff;
    uint32_t ngroups;
    const uint32_t *unit_head;   // 1: unit has a head hit
    int32_t S, nnc;
    const int32_t *nc;
    const uint8_t *is_control;
    const double *coef;
    int32_t ncoef;
    const double *kern;
    int32_t bw;
    int32_t nondir;
    double region_thr, kurt_thr, corr_thr, hit_thr;
    int32_t want_corr;
    uint32_t *resync;            // per unit: 0 untouched, X, or 0xFFFFFFFF
    up_region *out;
    uint32_t *out_counts;
    uint32_t *nout;
    uint32_t out_cap;
    // scratch per workgroup slot (index = blockIdx.x)
    uint32_t *ring_hits;         // [2][W][S]
    double *reg_f, *reg_r;       // [2][reg_cap]
    uint32_t *reg_hit;           // [2][reg_cap] index into reg_hits or 0xFFFFFFFF
    uint32_t *reg_hits;          // [2][reg_cap][S]
    uint32_t reg_cap;
    uint32_t *err;               // nonzero: capacity exceeded / contract violated
    // whole-buffer replay (configurations outside the parallel scan: -r <= 0
    // makes the leap branch of processPosition live, quirk Q11; bw > kMaxBw):
    // every unit is replayed, never resynced
    int32_t replay_all;
    // the deque window: dynamic LDS (ring_lds) or, for very wide kernels,
    // global scratch [2][W] per array
    int32_t ring_lds;
    double *ring_f, *ring_r;
    uint8_t *ring_has;
    // every replayed region's stored scores (Region::scores, data.cpp:92-96),
    // f then r, for strandCorr(shift) in strand_shift: slab + per-region offset
    double *out_scores;
    uint64_t *out_score_off;     // [out_cap], ~0 when the slab was full
    unsigned long long *nscores;
    uint64_t scores_cap;
    // -w (density profile) of replayed units: every processPosition with a
    // nonzero score (peakcall.cpp:80-83) as (unit, event, pos, score), in
    // emission order per buffer; event = index of the unit's add() whose
    // retirement loop wrote it, or kFlushEvent for its flushContig()
    uint32_t *prof_unit, *prof_event, *prof_pos;  // null: not captured
    double *prof_score;
    unsigned long long *nprof;
    uint64_t prof_cap;
    // threshold <= 0 chains (run_q11): group g replays from its first unit
    // (its adds at >= gskip[g]: the start of that unit's last run) with a
    // fresh state, and stops after the first leap it processes -- outside
    // that first unit -- that closes the open region with a clean window
    // (no Q1 leftovers, every add aligned since the last full drain): from
    // there on K1q's records hold.  gstop[2g] / [2g + 1] = (unit, leap
    // position) or ~0 when the group ran to its end; out_group[slot] = the
    // group of each record
    int32_t q11;
    const uint32_t *gskip;
    uint32_t *gstop;
    uint32_t *out_group;
    // chains as ranges of one buffer's unit list (segmented replay): group g
    // walks gunits[gbeg[g] .. gend[g]) -- null: goff's ranges
    const uint32_t *gbeg, *gend;
};

constexpr uint32_t kFlushEvent = 0xFFFFFFFFu;

struct EmuState {
    // window: deque[j] = cell (head + j) % W
    double *rf, *rr;      // LDS
    uint8_t *rhas;        // LDS
    uint32_t *rhits;      // global [W][S]
    uint32_t W, head;
    uint32_t buffer_pos, last_pos;
    // open Region
    uint32_t left, n, peak_pos;
    double peak_score;
    double *gf, *gr;
    uint32_t *ghit, *ghits;
    uint32_t nhits;
    uint32_t cur_unit;
    uint32_t close_pos;   // position of the add being processed, 0 during a flush
    uint32_t ev;          // index of that add within the unit (kFlushEvent: the flush)
    bool aligned;
    uint64_t horizon;     // positions <= horizon may hold misaligned leftovers
    bool resynced;
    // q11 chains: the window holds only aligned adds since a full drain (or
    // a clean unit start); a leap may end the chain; where it did; the group
    bool clean, may_stop;
    uint32_t stop_pos, group;
};

__device__ static bool any_at(const EmuParams &P, uint32_t u, int strand, int s, uint64_t p) {
    return fld_at(track_u8(P.units[u], P.S, strand, s), (int64_t)p) != 0;
}

// Every lane of the wave runs the state machine on identical copies of
// EmuState (wave-uniform control flow); the loops over the window, the
// samples and a region's positions are split over the lanes, and every sum
// whose order the reference fixes is added up in that order from a stage of
// 64 per-lane terms in LDS (each lane reads the same broadcast values, so the
// copies stay identical).  Stores and atomics of a single value go through
// lane 0.
struct EmuLds {
    uint32_t counts[kMaxSamples];  // the current add's counts per sample
    double t0[64], t1[64], t2[64];
};

__device__ __forceinline__ void emu_sync() { __syncthreads(); }  // one wave per workgroup

// the 64 staged terms of a chunk of `m` positions, added in position order
__device__ __forceinline__ double emu_add_terms(double acc, const double *t, int m) {
    for (int k = 0; k < m; ++k) acc = acc + t[k];
    return acc;
}

__device__ __forceinline__ uint32_t emu_wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}

// processRegion (peakcall.cpp:33-53) + Region statistics, appended to out
__device__ static void emu_region(const EmuParams &P, EmuState &E, EmuLds &L) {
    const int S = P.S;
    const int lane = threadIdx.x;
    emu_sync();  // the region's positions and hit vectors, stored by other lanes
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(P.nout, 1u);
    slot = (uint32_t)__shfl((int)slot, 0);
    const bool keep = slot < P.out_cap;
    if (!keep && lane == 0) atomicOr(P.err, 2u);
    const uint32_t n = E.n;
    // exptSums per sample (integer sums: any order)
    uint32_t nonctl = 0, total = 0;
    for (int s = 0; s < S; ++s) {
        uint32_t part = 0;
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t h = E.ghit[i];
            if (h != 0xFFFFFFFFu) part += E.ghits[(uint64_t)h * S + s];
        }
        const uint32_t acc = emu_wave_sum(part);
        if (!P.is_control[s]) nonctl += acc;
        total += acc;
        if (keep && lane == (s & 63)) P.out_counts[(uint64_t)slot * S + s] = acc;
    }
    // posMean / posKurtosis with a UShort position index (data.cpp:133-182):
    // count and psum are integer sums; sum2 and sum4 in position order
    auto pooled = [&](uint32_t i) -> uint32_t {
        const uint32_t h = E.ghit[i];
        if (h == 0xFFFFFFFFu) return 0u;
        uint32_t pc = 0;
        for (int s = 0; s < S; ++s) pc += E.ghits[(uint64_t)h * S + s];
        return pc;
    };
    uint32_t cpart = 0, ppart = 0;
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t pc = pooled(i);
        cpart += pc;
        ppart += pc * (uint32_t)(uint16_t)i;
    }
    const uint32_t count = emu_wave_sum(cpart), psum = emu_wave_sum(ppart);
    const double x_bar = (double)psum / (double)count;
    double sum2 = 0.0, sum4 = 0.0;
    for (uint32_t b = 0; b < n; b += 64) {
        const uint32_t i = b + lane;
        double a2 = 0.0, a4 = 0.0;
        if (i < n) {
            const uint32_t pc = pooled(i);
            if (pc != 0u || E.ghit[i] != 0xFFFFFFFFu) {  // a stored hit (exptSums may be 0)
                const double d = (double)(uint16_t)i - x_bar;
                const double d2 = d * d;
                a2 = (double)pc * d2;
                a4 = (double)pc * (d2 * d2);
            }
        }
        L.t0[lane] = a2;
        L.t1[lane] = a4;
        emu_sync();
        const int m = n - b < 64 ? (int)(n - b) : 64;
        // positions without a stored hit add nothing in the reference; a
        // +0.0 here leaves the (non-negative) sums as they are
        sum2 = emu_add_terms(sum2, L.t0, m);
        sum4 = emu_add_terms(sum4, L.t1, m);
        emu_sync();
    }
    const double kurt = ((double)count - 1) * sum4 / (sum2 * sum2);
    double corr = __builtin_nan("");
    if (P.want_corr && n > 3) {
        double s1 = 0.0, s2 = 0.0;
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            L.t0[lane] = i < n ? E.gf[i] : 0.0;
            L.t1[lane] = i < n ? E.gr[i] : 0.0;
            emu_sync();
            const int m = n - b < 64 ? (int)(n - b) : 64;
            s1 = emu_add_terms(s1, L.t0, m);
            s2 = emu_add_terms(s2, L.t1, m);
            emu_sync();
        }
        const double m1 = s1 / (double)n, m2 = s2 / (double)n;
        double q1 = 0.0, q2 = 0.0, q3 = 0.0;
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            double d1 = 0.0, d2 = 0.0;
            if (i < n) {
                d1 = E.gf[i] - m1;
                d2 = E.gr[i] - m2;
            }
            L.t0[lane] = d1 * d1;
            L.t1[lane] = d2 * d2;
            L.t2[lane] = d1 * d2;
            emu_sync();
            const int m = n - b < 64 ? (int)(n - b) : 64;
            q1 = emu_add_terms(q1, L.t0, m);
            q2 = emu_add_terms(q2, L.t1, m);
            q3 = emu_add_terms(q3, L.t2, m);
            emu_sync();
        }
        const double sd1 = sqrt(q1 / ((double)n - 1)), sd2 = sqrt(q2 / ((double)n - 1));
        corr = q3 / (((double)n - 1) * sd1 * sd2);
    }
    bool acc = (double)nonctl >= P.hit_thr;
    if (acc) acc = P.kurt_thr == 0 || (n > 1 && kurt <= P.kurt_thr);
    if (acc) acc = P.corr_thr <= -1 || corr >= P.corr_thr;
    if (keep && P.out_scores) {
        unsigned long long off = 0;
        if (lane == 0) off = atomicAdd(P.nscores, 2ull * n);
        off = (unsigned long long)__shfl((long long)off, 0);
        if (off + 2ull * n <= P.scores_cap) {
            for (uint32_t i = lane; i < n; i += 64) {
                P.out_scores[off + i] = E.gf[i];
                P.out_scores[off + n + i] = E.gr[i];
            }
            if (lane == 0) P.out_score_off[slot] = off;
        } else if (lane == 0) {
            P.out_score_off[slot] = ~0ull;
            atomicOr(P.err, 8u);
        }
    }
    if (keep && lane == 0) {
        if (P.out_group) P.out_group[slot] = E.group;
        up_region &o = P.out[slot];
        o.unit = E.cur_unit;
        o.left = E.left;
        o.right = E.left + n - 1;
        o.peak = E.peak_pos;
        o.sum = total;
        o.nonctl_sum = nonctl;
        o.accepted = acc;
        o.close_pos = E.close_pos;
        o.peak_score = E.peak_score;
        o.kurtosis = kurt;
        o.corr = corr;
    }
    E.left = 0;
    E.n = 0;
    E.nhits = 0;
    E.peak_pos = 0;
    E.peak_score = 0.0;
}

// Region::addPos (data.cpp:92-102); hits (cell index or none) are copied
__device__ static void emu_addpos(const EmuParams &P, EmuState &E, int cell, double f, double r) {
    const int lane = threadIdx.x;
    if (E.n >= P.reg_cap) {
        if (lane == 0) atomicOr(P.err, 1u);
        return;
    }
    if (lane == 0) {
        E.gf[E.n] = f;
        E.gr[E.n] = r;
        E.ghit[E.n] = cell >= 0 ? E.nhits : 0xFFFFFFFFu;
    }
    if (cell >= 0) {
        const uint32_t h = E.nhits++;
        // lane s % 64 wrote the cell's count of sample s (emu_add)
        for (int s = lane; s < P.S; s += 64) E.ghits[(uint64_t)h * P.S + s] = E.rhits[(uint64_t)cell * P.S + s];
    }
    E.n++;
    const double score = f + r;
    if (E.peak_pos == 0 || score > E.peak_score) {
        E.peak_pos = E.left + E.n - 1;
        E.peak_score = score;
    }
}

// processPosition (peakcall.cpp:55-86) of the front cell
__device__ static void emu_process(const EmuParams &P, EmuState &E, EmuLds &L, uint32_t pos, int cell) {
    const int lane = threadIdx.x;
    if (!(pos > E.last_pos) && lane == 0) atomicOr(P.err, 4u);
    const double f = E.rf[cell], r = E.rr[cell];
    const int hc = E.rhas[cell] ? cell : -1;
    const double score = f + r;
    // q11 chain end: a leap that closes the open region (left set, or
    // nothing open) over a clean window
    const bool stop = P.q11 && E.may_stop && pos != E.last_pos + 1 && E.clean && (E.left != 0 || E.n == 0);
    if (pos == E.last_pos + 1) {
        if (E.left != 0) {
            if (score >= P.region_thr) emu_addpos(P, E, hc, f, r);
            else emu_region(P, E, L);
        } else if (score >= P.region_thr) {
            E.left = pos;
            emu_addpos(P, E, hc, f, r);
        }
    } else {
        if (E.left != 0) emu_region(P, E, L);
        if (score >= P.region_thr) emu_addpos(P, E, hc, f, r);
    }
    if (P.prof_score && score != 0.0 && !stop && lane == 0) {  // profileOut_->write(PosScore(...)), peakcall.cpp:80-83
        const unsigned long long k = atomicAdd(P.nprof, 1ull);
        if (k < P.prof_cap) {
            P.prof_unit[k] = E.cur_unit;
            P.prof_event[k] = E.ev;
            P.prof_pos[k] = pos;
            P.prof_score[k] = score;
        } else {
            atomicOr(P.err, 16u);
        }
    }
    E.last_pos = pos;
    // resync: aligned, leftovers retired, nothing open
    if (!P.replay_all && E.aligned && (uint64_t)pos > E.horizon && E.n == 0) E.resynced = true;
    if (stop) {
        E.resynced = true;
        E.stop_pos = pos;
    }
    E.may_stop = true;  // (a chain's own first position is a leap from its fresh state)
}

// ProfileBuffer::add (peakcall.cpp:161-222) without the contig switch; the
// add's counts are in L.counts (with_counts) -- none for a flush
__device__ static void emu_add(const EmuParams &P, EmuState &E, EmuLds &L, bool with_counts, uint32_t pos,
                               bool forward) {
    const int lane = threadIdx.x;
    uint16_t n_static = (uint16_t)E.W;
    if (pos <= E.buffer_pos + 2u * (uint32_t)P.bw) n_static = (uint16_t)(pos - E.buffer_pos);
    if (E.buffer_pos != 0) {
        for (uint16_t i = 0; i < n_static && !E.resynced; ++i) {
            if (E.buffer_pos + i > (uint32_t)P.bw) {
                const int cell = (int)E.head;
                emu_process(P, E, L, E.buffer_pos + i - P.bw, cell);
                if (lane == 0) {
                    E.rf[cell] = 0.0;
                    E.rr[cell] = 0.0;
                    E.rhas[cell] = 0;
                }
                E.head = (E.head + 1) % E.W;
            }
        }
        if (E.buffer_pos > (uint32_t)P.bw && n_static == E.W) E.clean = true;  // every cell retired
    } else if (pos <= (uint32_t)P.bw) {
        E.clean = false;  // quirk Q1: the unit's first add lands misaligned
    }
    if (E.resynced) return;
    double cs = 0.0;
    if (with_counts) {  // countSum in the reference's sample order (uniform: LDS broadcasts)
        if (P.ncoef == 0) {
            for (int s = 0; s < P.S; ++s)
                if (!P.is_control[s]) cs = cs + (double)L.counts[s];
        } else {
            int k = 0;
            for (int s = 0; s < P.S && k < P.ncoef; ++s)
                if (!P.is_control[s]) { cs = cs + (double)L.counts[s] * P.coef[k]; ++k; }
            for (int s = 0; s < P.S; ++s)
                if (!P.is_control[s]) cs = cs + (double)L.counts[s];
        }
    }
    emu_sync();  // the retired cells' clears before the window's update
    if (cs != 0.0) {
        // each cell gains its kernel term once per add: split over the lanes
        for (uint32_t j = lane; j < E.W; j += 64) {
            const uint32_t c = (E.head + j) % E.W;
            if (forward) E.rf[c] = E.rf[c] + P.kern[j] * cs;
            else E.rr[c] = E.rr[c] + P.kern[j] * cs;
        }
        const uint32_t c = (E.head + P.bw) % E.W;
        const bool had = E.rhas[c] != 0;
        for (int s = lane; s < P.S; s += 64) {
            if (had) E.rhits[(uint64_t)c * P.S + s] += L.counts[s];
            else E.rhits[(uint64_t)c * P.S + s] = L.counts[s];
        }
        emu_sync();  // every lane has read rhas[c]
        if (lane == 0) E.rhas[c] = 1;
        emu_sync();  // the window as the next retirements read it
    }
    E.buffer_pos = pos;
}

__global__ void __launch_bounds__(64) emulate_kernel(EmuParams P) {
    extern __shared__ double emu_lds[];  // the window when P.ring_lds: rf[W], rr[W], rhas[W]
    __shared__ EmuLds L;
    const int lane = threadIdx.x;
    const int buffer = blockIdx.x;  // scratch slot
    const int S = P.S;
    EmuState E;
    E.W = 2 * P.bw + 1;
    if (P.ring_lds) {
        E.rf = emu_lds;
        E.rr = emu_lds + E.W;
        E.rhas = (uint8_t *)(emu_lds + 2 * E.W);
    } else {
        E.rf = P.ring_f + (uint64_t)buffer * E.W;
        E.rr = P.ring_r + (uint64_t)buffer * E.W;
        E.rhas = P.ring_has + (uint64_t)buffer * E.W;
    }
    double *rf = E.rf, *rr = E.rr;
    uint8_t *rhas = E.rhas;
    E.rhits = P.ring_hits + (uint64_t)buffer * E.W * S;
    E.gf = P.reg_f + (uint64_t)buffer * P.reg_cap;
    E.gr = P.reg_r + (uint64_t)buffer * P.reg_cap;
    E.ghit = P.reg_hit + (uint64_t)buffer * P.reg_cap;
    E.ghits = P.reg_hits + (uint64_t)buffer * P.reg_cap * S;
    E.group = 0;
    E.clean = true;
    E.may_stop = true;
    E.stop_pos = 0;

    for (uint32_t g = blockIdx.x; g < P.ngroups; g += gridDim.x) {
    bool in_chain = false;
    if (P.q11) {
        if (lane == 0) {
            P.gstop[2 * g] = 0xFFFFFFFFu;
            P.gstop[2 * g + 1] = 0xFFFFFFFFu;
        }
        E.group = g;
        E.clean = true;
    }
    const uint32_t gk0 = P.gbeg ? P.gbeg[g] : P.goff[g], gk1 = P.gbeg ? P.gend[g] : P.goff[g + 1];
    for (uint32_t gk = gk0; gk < gk1; ++gk) {
        const uint32_t u = P.gunits[gk];
        // q11 chains start at their group's first unit and end for good
        const bool q11_first = P.q11 && gk == gk0;
        if (P.q11 && !in_chain && !q11_first) break;
        if (!in_chain) {
            if (!q11_first && !P.unit_head[u]) continue;
            // chain start: fresh buffer state (the previous unit ended clean)
            for (uint32_t j = lane; j < E.W; j += 64) { rf[j] = 0.0; rr[j] = 0.0; rhas[j] = 0; }
            emu_sync();
            E.head = 0;
            E.buffer_pos = 0;
            E.last_pos = 0;
            E.left = 0;
            E.n = 0;
            E.nhits = 0;
            E.peak_pos = 0;
            E.peak_score = 0.0;
            E.may_stop = false;
            in_chain = true;
        }
        uint32_t nadd = 0;  // add() calls of this unit so far
        E.cur_unit = u;  // contig switch relabels the open region (peakcall.cpp:164-168)
        E.aligned = false;
        E.horizon = ~0ull;
        E.resynced = false;
        const UnitDesc U = P.units[u];
        const int nstr = U.nstrands;
        const uint64_t from = q11_first ? P.gskip[g] : 1;
        // walk the unit's add() positions in order, 64 at a time
        for (uint64_t base = from; base <= U.len && !E.resynced; base += 64) {
            const uint64_t p = base + lane;
            uint32_t any0 = 0, any1 = 0;
            if (p <= U.len) {
                for (int s = 0; s < S; ++s) {
                    any0 |= any_at(P, u, 0, s, p) ? 1u : 0u;
                    if (nstr == 2) any1 |= any_at(P, u, 1, s, p) ? 1u : 0u;
                }
            }
            const uint64_t m0 = __ballot(any0 != 0), m1 = __ballot(any1 != 0);
            uint64_t m = m0 | m1;
            while (m && !E.resynced) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const uint32_t pos = (uint32_t)(base + b);
                for (int st = 0; st < 2 && !E.resynced; ++st) {
                    if (!(((st ? m1 : m0) >> b) & 1)) continue;
                    for (int s = lane; s < S; s += 64) L.counts[s] = count_at(U, S, nstr == 2 ? st : 0, s, pos);
                    emu_sync();
                    E.close_pos = pos;
                    E.ev = nadd++;
                    const bool first_aligned = !E.aligned && pos > (uint32_t)P.bw;
                    emu_add(P, E, L, true, pos, nstr == 2 ? st == 0 : P.unit_buffer[u] == 0);
                    if (first_aligned) {
                        E.aligned = true;
                        E.horizon = (uint64_t)pos + P.bw;
                    }
                    emu_sync();  // L.counts is rewritten by the next add
                }
            }
        }
        bool stop = false;
        if (E.resynced) {
            if (lane == 0) P.resync[u] = E.last_pos + 1;
        } else {
            // explicit flushContig() at the end of the unit's pass
            E.close_pos = 0;
            E.ev = kFlushEvent;
            emu_add(P, E, L, false, E.buffer_pos + E.W, true);
            E.buffer_pos = 0;
            E.last_pos = 0;
            if (lane == 0) P.resync[u] = 0xFFFFFFFFu;
            emu_sync();
            bool dirty = false;
            for (uint32_t j = lane; j < E.W; j += 64) dirty |= rf[j] != 0.0 || rr[j] != 0.0 || rhas[j] != 0;
            const bool win = __ballot(dirty) == 0;
            E.clean = win;
            // a q11 chain carries its open region on: only a leap ends it
            stop = !P.q11 && win && E.n == 0;
        }
        if (E.resynced) {
            stop = true;
            if (P.q11 && lane == 0) {
                P.gstop[2 * g] = u;
                P.gstop[2 * g + 1] = E.stop_pos;
            }
        }
        if (stop) in_chain = false;
        emu_sync();
    }
    }  // groups
}

// Run starts of every unit for the segmented replay: the adds a with no add
// in [a - 2bw - 1, a - 1] of the same unit (any track: every sample, both
// strands).  At such an add the window drains completely, so a replay that
// starts there from a fresh state is exact from its first retirement on
// (api.hip run_replay).  One wave per strip: presence words of the strip, the
// last add before it searched backwards (up to 2bw + 1 positions), previous
// adds by prefix-max scans; the starts are appended as (unit << 32 | pos).
__global__ void __launch_bounds__(256) leap_adds_kernel(const UnitDesc *units, uint32_t nunits,
                                                        uint32_t nstrips, int S, int bw,
                                                        unsigned long long *out, uint32_t *count,
                                                        uint32_t cap) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    const int64_t gap = 2 * (int64_t)bw + 1;
    constexpr int64_t kNone = -((int64_t)1 << 40);
    for (uint32_t strip = wave; strip < nstrips; strip += nwaves) {
        const uint32_t u = find_unit(units, nunits, strip);
        const UnitDesc U = units[u];
        const int64_t p0 = 1 + (int64_t)(strip - U.strip0) * kStrip;
        if (p0 > (int64_t)U.len) continue;
        auto word_bits = [&](int64_t wbase) -> uint64_t {  // adds at wbase .. wbase + 63 (within 1..len)
            uint64_t m = 0;
            if (wbase + 63 < 1 || wbase > (int64_t)U.len) return 0;
            for (int st = 0; st < U.nstrands; ++st)
                for (int k = 0; k < S; ++k) {
                    const int64_t n0 = kPadPos + wbase - 1;
                    gu8 *t = track_u8(U, S, st, k) + fbyte(n0);
                    const uint32_t sh = fshift(n0);
                    // 64 fields from 16 bytes (aligned: wbase - 1 is a multiple of 64)
                    const u32x4 x = *(gu32x4 *)t;
                    (void)sh;
                    m |= nz_bits64(x);
                }
            if (wbase < 1) m &= ~0ull << (1 - wbase);
            if (wbase + 63 > (int64_t)U.len) m &= (U.len - wbase + 1) >= 64 ? ~0ull : ((1ull << (U.len - wbase + 1)) - 1);
            return m;
        };
        // the last add before the strip, within gap positions of it
        int64_t carry = kNone;
        for (int64_t back = 0; back < gap; back += 64 * 64) {
            const int64_t wb = p0 - 64 - back - 64 * lane;  // lane's word, going backwards
            uint64_t m = 0;
            if (wb + 63 >= p0 - gap && wb + 63 >= 1) m = word_bits(wb);
            int64_t v = m ? wb + 63 - __builtin_clzll(m) : kNone;
            if (v < p0 - gap) v = kNone;
            for (int o = 32; o > 0; o >>= 1) {
                const int64_t y = __shfl_xor((long long)v, o);
                v = y > v ? y : v;
            }
            if (v != kNone) { carry = v; break; }
        }
        for (int r = 0; r < kStripWords / 64; ++r) {
            const int64_t wbase = p0 + 64 * (64 * r + lane);
            const uint64_t m = word_bits(wbase);
            // previous add before this lane's word: carry, or the highest add
            // of the earlier words of this round (exclusive prefix max)
            int64_t v = m ? wbase + 63 - __builtin_clzll(m) : kNone;
            int64_t inc = v;
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t y = __shfl_up((long long)inc, d);
                if (lane >= d && y > inc) inc = y;
            }
            int64_t prev = __shfl_up((long long)inc, 1);
            if (lane == 0) prev = kNone;
            prev = prev > carry ? prev : carry;
            uint64_t mm = m;
            while (mm) {
                const int b = __builtin_ctzll(mm);
                mm &= mm - 1;
                const int64_t a = wbase + b;
                if (prev == kNone || a - prev > gap) {
                    const uint32_t k = atomicAdd(count, 1u);
                    if (k < cap) out[k] = ((unsigned long long)u << 32) | (uint32_t)a;
                }
                prev = a;
            }
            const int64_t top = __shfl((long long)inc, 63);
            carry = top > carry ? top : carry;
        }
    }
}

// a unit with an add() past bw cannot end its pass dirty (quirk Q1 leaks
// need every add at <= bw), so the buffer's next unit starts a new chain
// group.  One block per unit scans from bw + 1 until it finds a tag of any
// track (typically within a few hundred positions).
__global__ void __launch_bounds__(256) unit_aligned_kernel(const UnitDesc *units, int S, int bw, uint32_t *flag) {
    const UnitDesc U = units[blockIdx.x];
    for (uint64_t base = (uint64_t)bw + 1; base <= U.len; base += 4096) {
        bool any = false;
        for (int i = 0; i < 16; ++i) {
            const uint64_t p = base + (uint64_t)threadIdx.x * 16 + i;
            if (p > U.len) break;
            for (int st = 0; st < U.nstrands && !any; ++st)
                for (int k = 0; k < S && !any; ++k) any = fld_at(track_u8(U, S, st, k), (int64_t)p) != 0u;
        }
        if (__syncthreads_or(any)) {
            if (threadIdx.x == 0) flag[blockIdx.x] = 1u;
            return;
        }
    }
}

// head-hit detection: any pooled countSum != 0 at positions 1..bw
template <int POOL>
__device__ __forceinline__ void head_detect_unit(const UnitDesc *units, uint32_t unit, int S, int nnc,
                                                 const int32_t *nc, const double *coef, int bw,
                                                 uint32_t *head, uint32_t *mirror) {
    const UnitDesc U = units[unit];
    uint32_t hit = 0;
    for (int p = 1 + (int)threadIdx.x; p <= bw && (uint32_t)p <= U.len; p += blockDim.x) {
        for (int st = 0; st < U.nstrands; ++st) {
            double cs = 0.0;
            for (int k = 0; k < nnc; ++k) {
                const uint32_t c = count_at(U, S, st, nc[k], p);
                cs = POOL == 2 ? cs + (double)c * coef[k] : cs + (double)c;
            }
            if (POOL == 2)
                for (int k = 0; k < nnc; ++k) cs = cs + (double)count_at(U, S, st, nc[k], p);
            if (cs != 0.0) hit = 1;
        }
    }
    const uint32_t v = __syncthreads_or(hit) ? 1u : 0u;
    if (threadIdx.x == 0) {
        head[unit] = v;
        if (mirror) mirror[unit] = v;  // mapped host copy: no read-back copy
    }
}

// K2a with the head detection in its trailing blocks (one block per unit;
// its threads stride over positions 1..bw): one launch fewer per pass
template <int POOL>
__global__ void __launch_bounds__(kSegBlock) seg_count_head_kernel(
    const uint64_t *__restrict__ info, uint64_t *__restrict__ cnt, uint64_t *__restrict__ bsum,
    uint32_t n, uint32_t nsb, const UnitDesc *units, int S, int nnc, const int32_t *nc,
    const double *coef, int bw, uint32_t *head, uint32_t *mirror) {
    if (blockIdx.x >= nsb) {  // block-uniform
        head_detect_unit<POOL>(units, blockIdx.x - nsb, S, nnc, nc, coef, bw, head, mirror);
        return;
    }
    seg_count_block(info, cnt, bsum, n);
}

}  // namespace upk
