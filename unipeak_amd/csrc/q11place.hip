// unipeak_amd/csrc/q11place.hip -- the records of a K1q pass (threshold
// <= 0) in the reference's form, on the device.  #included by api.hip.
//
// K3 leaves one record per run of processed positions in K2's order (unit-
// major, position order) in a device stage.  The reference reports each of
// them differently (peakcall.cpp:55-86, 164-168; DESIGN.md §4a "K1q"):
// coordinates + 1 (the run was reached by a leap), and a unit's last run is
// still open after its flush, so the buffer's next unit with records
// relabels it and closes it first (UP_CLOSE_Q11_HEAD); the buffer's last
// run is never closed.  The per-unit edits of the head chains (q11_finish)
// drop K1q records where the exact replay's take over and leave slots for
// those.  Output order, per unit: [the moved-in record] [replayed records]
// [the unit's own kept records].
//
//   q11_table_kernel   one block: per unit its record range (binary search
//                      of K2's unit column), the previous / next unit with
//                      records in its buffer, kept range, output offset
//                      (block scans with a carry over chunks of units)
//   q11_scatter_kernel one thread per record: stage -> destination (the
//                      pinned mapped host records or the caller's target),
//                      plus each record's stored positions and source unit
//                      (up_shift_scan)

namespace upk {

constexpr uint32_t kQ11Full = 1u, kQ11NoMove = 2u;  // Q11Edit::flags
constexpr uint32_t kQ11None = 0xFFFFFFFFu;

// per unit, where its records go
struct Q11Place {
    uint64_t first;       // the unit's first record in K2's order
    uint64_t base;        // destination of its kept record jlo
    uint64_t moved_dest;  // destination of its last record (the buffer's next unit), ~0: dropped
    uint32_t cnt;         // its records
    uint32_t jlo, jhi;    // kept own records [jlo, jhi) (the last one is never an own record)
    uint32_t moved_unit;  // the unit the last record moves to
};

struct Q11Edit {     // per unit (null: no edits)
    uint32_t lo, hi;   // keep own records with lo <= start < hi (raw run starts)
    uint32_t nrep;     // replayed records placed after the moved-in one
    uint32_t flags;    // kQ11Full: no own records and no moved-in one; kQ11NoMove: no moved-in one
};

// lower bound of v in a[lo, hi)
__device__ __forceinline__ uint64_t lb_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint32_t v) {
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// inclusive block scan (sum) of one value per thread, blockDim 1024
__device__ uint64_t block_incl_sum(uint64_t v, uint64_t *sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = (uint64_t)__shfl_up((long long)v, o);
        if (lane >= o) v += y;
    }
    if (lane == 63) sh[w] = v;
    __syncthreads();
    uint64_t before = 0;
    for (int k = 0; k < w; ++k) before += sh[k];
    __syncthreads();
    return v + before;
}

// suffix minimum (over threads t' >= t) of one value per thread, blockDim 1024
__device__ uint32_t block_suffix_min(uint32_t v, uint32_t *sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_down((int)v, o);
        if (lane + o < 64 && y < v) v = y;
    }
    if (lane == 0) sh[w] = v;
    __syncthreads();
    for (int k = w + 1; k < 16; ++k) v = sh[k] < v ? sh[k] : v;
    __syncthreads();
    return v;
}

// scratch per unit: [0] output offset, [1] moved-in flag | next unit << 32
__global__ void __launch_bounds__(1024) q11_table_kernel(const int32_t *__restrict__ ubuf, uint32_t nu,
                                                         const uint32_t *__restrict__ runit,
                                                         const uint32_t *__restrict__ starts,
                                                         const uint64_t *__restrict__ nreg_p,
                                                         const Q11Edit *__restrict__ edit, Q11Place *tab,
                                                         uint64_t *scratch, unsigned long long *status,
                                                         unsigned long long *target_hdr, uint64_t dest_cap) {
    __shared__ uint64_t sh64[16];
    __shared__ uint32_t sh32[16];
    __shared__ uint32_t first_with[2];
    __shared__ uint32_t ex0[1025], ex1[1025];  // suffix minima of a chunk, [1024] = the carry
    __shared__ uint64_t chunk_tot;
    const uint64_t nreg = *nreg_p;
    const uint32_t t = threadIdx.x;
    if (t < 2) first_with[t] = kQ11None;
    __syncthreads();
    // A: each unit's record range; the first unit with records of each buffer
    for (uint32_t u = t; u < nu; u += blockDim.x) {
        const uint64_t f = lb_u32(runit, 0, nreg, u);
        const uint64_t e = lb_u32(runit, f, nreg, u + 1);
        tab[u].first = f;
        tab[u].cnt = (uint32_t)(e - f);
        if (e > f) atomicMin(&first_with[ubuf[u] & 1], u);
    }
    __syncthreads();
    // B: the next unit with records in the same buffer (suffix minima, chunks
    // from the end with a carry per buffer)
    uint32_t carry0 = kQ11None, carry1 = kQ11None;
    const uint32_t nchunks = (nu + 1023) / 1024;
    for (uint32_t ch = nchunks; ch-- > 0;) {
        const uint32_t u = ch * 1024 + t;
        const bool in = u < nu;
        const bool has = in && tab[u].cnt != 0;
        const int b = in ? (ubuf[u] & 1) : 0;
        // exclusive: units after u -> shift by one thread
        const uint32_t v0 = has && b == 0 ? u : kQ11None, v1 = has && b == 1 ? u : kQ11None;
        uint32_t s0 = block_suffix_min(v0, sh32), s1 = block_suffix_min(v1, sh32);
        // s_b now covers t' >= t; the exclusive value is the inclusive one of t + 1
        ex0[t] = s0;
        ex1[t] = s1;
        if (t == 0) { ex0[1024] = carry0; ex1[1024] = carry1; }
        __syncthreads();
        uint32_t n0 = ex0[t + 1], n1 = ex1[t + 1];
        if (t + 1 < 1024) {
            n0 = n0 < carry0 ? n0 : carry0;
            n1 = n1 < carry1 ? n1 : carry1;
        }
        if (in) {
            const uint32_t nx = b == 0 ? n0 : n1;
            const bool prev = first_with[b] < u;
            const Q11Edit E = edit ? edit[u] : Q11Edit{0u, 0xFFFFFFFFu, 0u, 0u};
            const bool mv = has && prev && !(E.flags & (kQ11Full | kQ11NoMove));
            scratch[2 * u + 1] = (uint64_t)(mv ? 1u : 0u) | ((uint64_t)nx << 32);
        }
        const uint32_t c0 = ex0[0], c1 = ex1[0];
        __syncthreads();
        carry0 = c0 < carry0 ? c0 : carry0;
        carry1 = c1 < carry1 ? c1 : carry1;
    }
    __syncthreads();
    // C: kept range, output count, offsets (prefix sums with a carry)
    uint64_t base = 0;
    for (uint32_t ch = 0; ch < nchunks; ++ch) {
        const uint32_t u = ch * 1024 + t;
        uint64_t cnt = 0;
        if (u < nu) {
            const Q11Place T = tab[u];
            const Q11Edit E = edit ? edit[u] : Q11Edit{0u, 0xFFFFFFFFu, 0u, 0u};
            uint32_t jlo = 0, jhi = 0;
            if (T.cnt > 1 && !(E.flags & kQ11Full)) {  // own records: all but the last
                const uint64_t a = T.first, z = T.first + T.cnt - 1;
                jlo = (uint32_t)(lb_u32(starts, a, z, E.lo) - a);
                jhi = E.hi == 0xFFFFFFFFu ? (uint32_t)(z - a) : (uint32_t)(lb_u32(starts, a, z, E.hi) - a);
                if (jhi < jlo) jhi = jlo;
            }
            tab[u].jlo = jlo;
            tab[u].jhi = jhi;
            cnt = (scratch[2 * u + 1] & 1u) + E.nrep + (jhi - jlo);
        }
        const uint64_t inc = block_incl_sum(cnt, sh64);
        if (u < nu) scratch[2 * u] = base + inc - cnt;
        if (t == 1023) chunk_tot = inc;  // the chunk's total
        __syncthreads();
        base += chunk_tot;
        __syncthreads();
    }
    // D: bases and the moved record's destination
    for (uint32_t u = t; u < nu; u += blockDim.x) {
        const uint64_t s1 = scratch[2 * u + 1];
        const uint32_t nx = (uint32_t)(s1 >> 32);
        const Q11Edit E = edit ? edit[u] : Q11Edit{0u, 0xFFFFFFFFu, 0u, 0u};
        tab[u].base = scratch[2 * u] + (s1 & 1u) + E.nrep;
        uint64_t md = ~0ull;
        uint32_t mu = kQ11None;
        if (nx != kQ11None && (scratch[2 * nx + 1] & 1u)) {
            md = scratch[2 * nx];
            mu = nx;
        }
        tab[u].moved_dest = md;
        tab[u].moved_unit = mu;
    }
    if (t == 0) {
        const bool ok = base <= dest_cap;
        status[3] = base + 1;  // the output count (+1: written)
        if (target_hdr) *target_hdr = ok && nreg ? base : 0;
    }
}

// stage (K3's records and exptSums, K2's order) -> the destination; each
// record's stored positions (start, end) and source unit for up_shift_scan
__global__ void __launch_bounds__(256) q11_scatter_kernel(const up_region *__restrict__ stage,
                                                          const uint32_t *__restrict__ stage_counts,
                                                          const uint64_t *__restrict__ nreg_p, int S,
                                                          const Q11Place *__restrict__ tab, up_region *out,
                                                          uint32_t *out_counts, uint64_t dest_cap,
                                                          uint32_t *sh_start, uint32_t *sh_end,
                                                          uint32_t *sh_unit) {
    const uint64_t nreg = *nreg_p;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreg;
         i += (uint64_t)gridDim.x * blockDim.x) {
        up_region r = stage[i];
        const uint32_t u = r.unit;
        const Q11Place T = tab[u];
        const uint64_t j = i - T.first;
        uint64_t d;
        if (j + 1 < T.cnt) {
            if (j < T.jlo || j >= T.jhi) continue;
            d = T.base + (j - T.jlo);
            r.close_pos = UP_CLOSE_Q11;
        } else {
            if (T.moved_dest == ~0ull) continue;  // the buffer's last run: never closed
            d = T.moved_dest;
            r.unit = T.moved_unit;
            r.close_pos = UP_CLOSE_Q11_HEAD;
        }
        if (d >= dest_cap) continue;  // the host grows the area and reruns
        sh_start[d] = r.left;
        sh_end[d] = r.right;
        sh_unit[d] = u;
        r.left += 1;
        r.right += 1;
        r.peak += 1;
        out[d] = r;
        for (int s = 0; s < S; ++s) out_counts[d * S + s] = stage_counts[i * S + s];
    }
}

}  // namespace upk
