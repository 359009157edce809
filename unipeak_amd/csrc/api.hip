// unipeak_amd/csrc/api.hip -- C-ABI implementation (include/unipeak_hip.h):
// device memory for the unit tracks, kernel launches and the glue between
// them.  Host-side only; kernels live in kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <unordered_map>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/unipeak_hip.h"
#include "kernels.h"

#include "kernels.hip"  // device code shared with the per-NH units (nh_tu.hip)
#include "stats1.hip"   // (its LDS size)
#include "emulate.hip"
#include "q11place.hip"
#include "wide.hip"

namespace upk {
// the templated K1 / K3 / K4 kernels live in four translation units, one per
// window width NH (nh_tu.hip, built in parallel); these return their addresses
const void *scan_kernel_nh1(int, bool, bool, int);
const void *scan_kernel_nh2(int, bool, bool, int);
const void *scan_kernel_nh3(int, bool, bool, int);
const void *scan_kernel_nh4(int, bool, bool, int);
const void *scan_kernel_nh5(int, bool, bool, int);
const void *scan_kernel_nh6(int, bool, bool, int);
const void *scan_kernel_nh7(int, bool, bool, int);
const void *scan_kernel_nh8(int, bool, bool, int);
const void *stats_kernel_nh1(int, bool, int);
const void *stats_kernel_nh2(int, bool, int);
const void *stats_kernel_nh3(int, bool, int);
const void *stats_kernel_nh4(int, bool, int);
const void *stats_kernel_nh5(int, bool, int);
const void *stats_kernel_nh6(int, bool, int);
const void *stats_kernel_nh7(int, bool, int);
const void *stats_kernel_nh8(int, bool, int);
const void *shift_kernel_nh1(int);
const void *shift_kernel_nh2(int);
const void *shift_kernel_nh3(int);
const void *shift_kernel_nh4(int);
const void *shift_kernel_nh5(int);
const void *shift_kernel_nh6(int);
const void *shift_kernel_nh7(int);
const void *shift_kernel_nh8(int);
// window words on each side of an output word: ceil((bw + 1) / 64)
static int window_nh(int bw) { return (bw + 64) / 64; }
static const void *scan_kernel_for(int bw, int pool, bool nd, bool prof, int mode) {
    switch (window_nh(bw)) {
    case 1: return scan_kernel_nh1(pool, nd, prof, mode);
    case 2: return scan_kernel_nh2(pool, nd, prof, mode);
    case 3: return scan_kernel_nh3(pool, nd, prof, mode);
    case 4: return scan_kernel_nh4(pool, nd, prof, mode);
    case 5: return scan_kernel_nh5(pool, nd, prof, mode);
    case 6: return scan_kernel_nh6(pool, nd, prof, mode);
    case 7: return scan_kernel_nh7(pool, nd, prof, mode);
    default: return scan_kernel_nh8(pool, nd, prof, mode);
    }
}
static const void *stats_kernel_for(int bw, int pool, bool nd, int one) {
    switch (window_nh(bw)) {
    case 1: return stats_kernel_nh1(pool, nd, one);
    case 2: return stats_kernel_nh2(pool, nd, one);
    case 3: return stats_kernel_nh3(pool, nd, one);
    case 4: return stats_kernel_nh4(pool, nd, one);
    case 5: return stats_kernel_nh5(pool, nd, one);
    case 6: return stats_kernel_nh6(pool, nd, one);
    case 7: return stats_kernel_nh7(pool, nd, one);
    default: return stats_kernel_nh8(pool, nd, one);
    }
}
static const void *shift_kernel_for(int bw, int pool) {
    switch (window_nh(bw)) {
    case 1: return shift_kernel_nh1(pool);
    case 2: return shift_kernel_nh2(pool);
    case 3: return shift_kernel_nh3(pool);
    case 4: return shift_kernel_nh4(pool);
    case 5: return shift_kernel_nh5(pool);
    case 6: return shift_kernel_nh6(pool);
    case 7: return shift_kernel_nh7(pool);
    default: return shift_kernel_nh8(pool);
    }
}
}  // namespace upk

using namespace upk;

namespace {

struct Unit {
    uint32_t len = 0;
    int32_t nstrands = 1;
    int32_t buffer = 0;
    uint8_t *dptr = nullptr;   // 4-bit tracks (kernels.h)
    uint64_t stride = 0;       // bytes per track
    uint32_t nstrips = 0;
    uint32_t strip0 = 0;
    uint32_t last_override = 0;
    bool has_override = false;
    // counts >= kEsc per track: position -> count (authoritative copy)
    std::vector<std::map<uint32_t, uint32_t>> ovf;
    uint64_t *d_ovf = nullptr;     // uploaded entries, sorted by (track, pos)
    uint32_t *d_ovf_off = nullptr; // [ntracks + 1]
    uint32_t *d_ovf_tidx = nullptr;  // [ntracks][nblk] escape tile per block (kNoTile: none)
    uint8_t *d_ovf_tiles = nullptr;  // [ntiles][kOvfBlk]
    uint8_t *d_pct = nullptr;        // pooled count track (POOL 1; UnitDesc::pct)
    bool ovf_dirty = false;
    bool cs_dirty = false;     // a track changed: rebuild its chunk-sum plane (csum_kernel)
    bool pool_dirty = true;    // rebuild the unit's pooled plane (pool_kernel)
    uint32_t ovf_max = 0;          // largest escaped count of any track
    uint32_t pad_bw = 0;           // the widest kernel the track padding covers (unit_stride)
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        // growth is rare (first passes); a pipelined pass may still read p
        if (p) (void)hipDeviceSynchronize();
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        size_t cap = want < 16 ? 16 : want + want / 4;
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

// pinned, device-mapped host memory: kernels write results straight into it
// (coherent, so the writes are visible to the host once the stream syncs)
template <typename T>
struct HostBuf {
    T *p = nullptr;    // host address
    T *dev = nullptr;  // device address of the same memory
    size_t n = 0;
    hipError_t ensure(size_t want) {
        if (want <= n && p) return hipSuccess;
        if (p) (void)hipDeviceSynchronize();
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
        n = 0;
        size_t cap = want < 16 ? 16 : want + want / 4;
        hipError_t e = hipHostMalloc((void **)&p, cap * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return e;
        e = hipHostGetDevicePointer((void **)&dev, p, 0);
        if (e == hipSuccess) n = cap;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
        n = 0;
    }
};

constexpr int kSlots = UP_MAX_IN_FLIGHT;  // passes in flight at most (up_run_async)

}  // namespace

struct up_ctx {
    int dev = 0;
    int ncu = 0;                     // compute units of the device
    // K1a workgroups per CU (UNIPEAK_K1A_PER_CU; 0 = resident max): 3 with
    // the 2-bit tracks and the register pre-screen (hg19, same box, two
    // rounds: K1a alone 0.35 vs 0.44 ms at 2, bench 4,395 vs 4,265 Gbp/s)
    int k1a_per_cu = 3;
    int k1b_per_cu = 0;              // K1b workgroups per CU (UNIPEAK_K1B_PER_CU; 0 = resident)
    int k3_per_cu = 0;               // K3 workgroups per CU (UNIPEAK_K3_PER_CU; 0 = resident)
    bool k3_one = true;              // batched K3 for one directional sample (UNIPEAK_K3_ONE=0: off)
    bool use_graphs = true;          // passes as hipGraphs (UNIPEAK_GRAPHS=0: plain launches)
    // streams of the passes: every K1a on one high-priority stream (stream
    // order serialises them; as resources free up the dispatcher serves it
    // first), the rest of a pass on one of n_chain chain streams in turn, so
    // that many passes' K1x..K3 may overlap (bench.py raises
    // GPU_MAX_HW_QUEUES so no two of them share a hardware queue)
    hipStream_t k1a_stream = nullptr;
    hipStream_t chain[4] = {};
    // chain streams in use (UNIPEAK_CHAINS, 1..4): three -- hg19 configs[1],
    // same box, two alternating rounds: 4,832 / 4,755 Gbp/s vs 4,652 / 4,487
    // with two and 4,636 / 4,604 with four
    int n_chain = 3;
    uint64_t nlaunch = 0;
    hipStream_t stream = nullptr;
    bool have_params = false;
    up_params p{};
    std::vector<uint8_t> ctl;
    std::vector<double> coef, kern;
    std::vector<int32_t> nc;
    DevBuf<double> d_kern, d_coef;
    DevBuf<int32_t> d_nc;
    DevBuf<uint8_t> d_ctl;
    DevBuf<uint32_t> d_wscreen;
    uint32_t wskip = 0;
    float fw[kScrHalo + 1] = {};     // fine screen weights per chunk distance
    float fthr = 0.f;
    // K1b keys (ScanParams::qmode): score = alpha * Q * (1 +- q_delta)
    bool q_ok = false;               // weights proportional to bw^2 - d^2 within q_delta
    double q_alpha = 0.0, q_delta = 1.0;
    uint32_t qno = 0, qyes = 0;
    uint32_t ovf_max_all = 0;        // largest escaped count of any unit
    DevBuf<uint32_t> d_stage;          // dense uint32 staging for synth / pack
    DevBuf<unsigned long long> d_pack_ovf;
    DevBuf<uint32_t> d_pack_n;
    DevBuf<unsigned long long> d_dbg;
    std::vector<Unit> units;
    bool units_dirty = true;
    std::vector<uint32_t> pool_sig;  // non-control samples + screen weights the pooled planes hold
    DevBuf<UnitDesc> d_units;
    std::vector<UnitDesc> h_units;   // host copy of d_units
    // the per-dataset index (chunk-sum planes, pooled planes, pooled count
    // tracks; DESIGN.md §3 "Index policy"): up_set_index_policy, whether the
    // unit table and the passes use it now, passes launched since the tracks
    // or the pooling last changed, builds so far
    int index_policy = UP_INDEX_AUTO;
    bool index_on = false;
    uint32_t passes_on_tracks = 0;
    uint64_t index_builds = 0;
    DevBuf<uint64_t> d_index_lists;  // sync_index's unit lists
    uint32_t nstrips = 0;
    int bw_layout = -1;  // bw the strip layout was computed for
    // per (track slot strand * S + sample, global strip): the strip or its
    // halo blocks hold an escape (ScanParams::esc, K1a's cheap bound)
    DevBuf<uint32_t> d_esc;
    uint32_t esc_nw = 0;
    DevBuf<uint32_t> d_unit_last;
    uint32_t k1a_waves = 0, k1a_xcap = 0;  // grid and per-wave stash size of the last K1a launch
    uint32_t ovf_cap = 256;
    uint64_t nreg = 0;
    bool ran = false;
    std::vector<uint32_t> unit_last;
    hipEvent_t ev[8] = {};
    double times[5] = {0, 0, 0, 0, 0};
    int timing = 2;                  // up_set_timing: 0 wall only, 1 + K1a, 2 every phase
    // passes in flight (up_run_async); slot = sequence % kSlots.  Each slot
    // owns its device buffers and its stream, so a pass's streaming K1a can
    // run while earlier passes' latency-bound K1b/K2/K3 finish (a pass's K1a
    // starts once the previous pass's K1a has ended, k1a_end); several slots
    // let the host enqueue passes while earlier ones are still completing
    struct Pass {
        hipStream_t stream = nullptr;
        hipEvent_t k1a_end = nullptr;   // this pass's K1a finished
        // K1x..K3 of the pass as hipGraphs, one per launch-argument set
        // (record targets rotate), most recent first
        std::vector<std::pair<std::vector<uint8_t>, hipGraphExec_t>> graphs;
        bool counters_armed = false;    // xcount / ovf_count are zero (re-armed by K2b)
        DevBuf<uint64_t> d_info;
        DevBuf<uint32_t> d_rec, d_ovf_count, d_ovf_rec, d_head;
        DevBuf<uint64_t> d_cnt, d_nreg, d_bsum;
        DevBuf<uint32_t> d_starts, d_ends, d_runit, d_peak_pos, d_xlist, d_xcount, d_xwcount, d_xref;
        DevBuf<double> d_peak_val;
        DevBuf<uint64_t> d_spk;          // K1 per-strip partial peaks (ScanParams::spk)
        DevBuf<double> d_corr;           // K3 (f, r) slabs for the strand correlation (-D -y)
        void release() {
            d_info.release(); d_rec.release(); d_ovf_count.release(); d_ovf_rec.release(); d_head.release();
            d_cnt.release(); d_nreg.release(); d_bsum.release(); d_starts.release(); d_ends.release();
            d_runit.release(); d_peak_pos.release(); d_xlist.release(); d_xcount.release();
            d_xwcount.release(); d_xref.release(); d_peak_val.release(); d_spk.release(); d_corr.release();
        }
        uint8_t *target = nullptr;   // record target of this pass (device address) or null
        void *target_hostp = nullptr;// host address of a host target
        uint64_t target_cap = 0;
        // what the caller set when it enqueued the pass (the launcher thread
        // launches it later): record target, timing level, K3 grid estimate
        uint8_t *req_target = nullptr;
        void *req_target_hostp = nullptr;
        uint64_t req_target_cap = 0, req_last_nreg = 0;
        uint64_t req_reg_cap = 0;    // record / overflow capacities: the caller's thread
        uint32_t req_ovf_cap = 0;    // grows them, the launcher thread only reads these
        int req_tl = 0;
        bool req_q11 = false;
        bool req_q11_place = false;  // the pass places its K1q records (q11_place)        // K1q instead of K1a/K1x/K1b (threshold <= 0, run_q11)
        bool lpending = false;       // queued for / being launched by the launcher thread
        int lrc = 0;                 // its launch result
        uint64_t cap = 0;            // reg_cap at launch
        uint32_t ovf_cap = 0;
        int tl = 0;                  // timing level at launch
        std::chrono::steady_clock::time_point t0;
        hipEvent_t ev[5] = {};       // K1a begin, K1a end, K1b end, K2 end, K3 end
        hipEvent_t done = nullptr;
    } pass[kSlots];
    uint64_t seq_launched = 0, seq_done = 0;
    int cur_slot = 0;                // slot of the last completed pass (host records)
    // Launcher thread: up_run_async hands the pass's HIP calls (K1a launch,
    // events, the K1x..K3 graph, ~40 us of host time) to it and returns, so
    // the caller's own per-step work overlaps them (at 8 GPUs a step is
    // ~0.1 ms and the host side bounds it).  UNIPEAK_LAUNCHER=0: launch on
    // the caller's thread.
    std::thread launcher;
    std::mutex lmu;
    std::condition_variable lcv;
    std::deque<int> lq;              // slots to launch, in order
    bool lbusy = false, lstop = false, use_launcher = true;
    // head-hit (quirk Q1) replay
    hipEvent_t host_work = nullptr;  // marks work on `stream` that a pass must follow
    DevBuf<uint32_t> d_resync, d_emu_n, d_emu_err, d_emu_counts, d_ring_hits, d_reg_hit, d_reg_hits;
    DevBuf<int32_t> d_unit_buffer;
    DevBuf<uint32_t> d_gunits, d_goff;  // K0 chain groups (emulate_units)
    DevBuf<uint32_t> d_gskip, d_gstop, d_emu_group;  // threshold <= 0 chains (Q11Chains)
    DevBuf<double> d_reg_f, d_reg_r;
    DevBuf<up_region> d_emu_out;
    DevBuf<double> d_ring_f, d_ring_r;   // K0 window in global memory (very wide kernels)
    // -w of replayed units (up_set_profile_capture): K0's nonzero
    // retirements, device buffers and the last run's host copy, per unit
    bool prof_capture = false;
    uint64_t pf_cap = 1u << 20;
    DevBuf<uint32_t> d_pf_unit, d_pf_event, d_pf_pos;
    DevBuf<double> d_pf_score;
    DevBuf<unsigned long long> d_pf_n;
    std::vector<uint32_t> h_pf_event, h_pf_pos;
    std::vector<double> h_pf_score;
    std::vector<uint64_t> h_pf_off;      // [units + 1]: each unit's slice of the h_pf_* arrays
    std::vector<uint32_t> h_resync;      // per unit: 0 not replayed, X resync, ~0 replayed to the end
    // K4 (up_shift_scan) buffers, kept across calls
    DevBuf<uint64_t> d_sh_idx, d_sh_off;
    DevBuf<double> d_sh_slab, d_sh_out;
    DevBuf<uint8_t> d_sh_pref;
    DevBuf<double> d_emu_scores;         // K0: stored scores of the replayed regions (f, r)
    DevBuf<uint64_t> d_emu_score_off;
    DevBuf<unsigned long long> d_emu_nscores;
    uint64_t emu_scores_cap = 1ull << 22;
    std::vector<uint64_t> h_score_off;   // per host region: offset in d_emu_scores or ~0
    DevBuf<uint8_t> d_ring_has;
    uint32_t emu_reg_cap = 1u << 18;     // K0: positions of one open region
    uint32_t emu_chain_reg_cap = 1u << 14;  // the same for chains (many slots at once)
    uint32_t seg_cap = 1u << 20;         // segmented replay: run starts
    DevBuf<unsigned long long> d_seg;
    DevBuf<uint32_t> d_seg_n, d_gbeg, d_gend;
    uint32_t emu_out_cap = 1u << 16;     // K0: region records
    bool host_regions = false;  // merged list lives on the host
    // threshold <= 0 through K1q (run_q11): the blocking pass in progress,
    // and per host record the unit whose tracks hold its positions (a region
    // closed in the buffer's next unit keeps the previous unit's positions)
    bool q11_run = false;
    DevBuf<uint32_t> d_q11_head;
    // K1q records finished on the device (q11place.hip): K3's stage, the
    // per-unit placement, the head chains' edits, and per placed record its
    // stored positions and source unit (up_shift_scan); q11_rep: the
    // replayed records among them (index, offset of their stored scores)
    bool q11_place_in_pass = false;  // the pass places its records itself (no heads)
    bool q11_placed = false;         // the current records are a placed K1q list
    // K0 chain groups: per unit, an add past bw (unit_aligned_kernel), kept
    // while the unit layout and the tracks are unchanged (sync_units clears it)
    std::vector<uint32_t> aligned_cache;
    bool aligned_valid = false;
    DevBuf<up_region> d_q11_stage;
    DevBuf<uint32_t> d_q11_stage_cnt;
    DevBuf<Q11Place> d_q11_tab;
    DevBuf<uint64_t> d_q11_scr;
    DevBuf<Q11Edit> d_q11_edit;
    DevBuf<uint32_t> d_q11_st, d_q11_en, d_q11_src;
    std::vector<std::pair<uint64_t, uint64_t>> q11_rep;
    std::vector<up_region> h_regions;
    std::vector<uint32_t> h_counts;
    std::vector<uint8_t> h_emulated;
    // per pass slot: head-hit flags (seg_count_head_kernel), host records, status
    HostBuf<uint32_t> hp_head[kSlots];
    HostBuf<up_region> hp_regions[kSlots];
    HostBuf<uint32_t> hp_counts[kSlots];
    HostBuf<unsigned long long> hp_status[kSlots];
    void *target_hostp = nullptr;    // host address of the current host target
    // up_unit_scatter staging: two mapped host buffers the scatter kernel
    // reads directly, reused once the event of their previous use fired
    HostBuf<uint32_t> hp_scat[2];
    hipEvent_t scat_ev[2] = {};
    int scat_i = 0;
    uint64_t reg_cap = 1u << 16;  // record capacity of one pass (grown on demand)
    uint8_t *target = nullptr;    // device address of the caller's record buffer
    uint64_t target_cap = 0;
    void *target_host = nullptr;  // host buffer we registered for it
    std::vector<void *> host_regs; // up_host_register ranges (unregistered at close)
    uint64_t last_nreg = 0;
};

static bool busy(const up_ctx *c) { return c && c->seq_launched != c->seq_done; }

// the tracks or the pooling changed: the index is rebuilt when a pass wants it
// (the per-unit dirty flags say what), and UP_INDEX_AUTO counts passes anew
static void index_stale(up_ctx *c) { c->passes_on_tracks = 0; }

// the context, K1a and chain streams idle
static void sync_all(up_ctx *c) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->k1a_stream);
    for (auto st : c->chain)
        if (st) (void)hipStreamSynchronize(st);
}

#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "unipeak_hip: %s failed: %s (%s:%d)\n", #x,             \
                    hipGetErrorString(e_), __FILE__, __LINE__);                     \
            return e_ == hipErrorOutOfMemory ? UP_E_NOMEM : UP_E_HIP;               \
        }                                                                           \
    } while (0)

// public entry points: C linkage comes from the declarations in
// include/unipeak_hip.h

int up_version(void) { return 10000; }
int up_track_bits(void) { return kTB; }

// K1a's stream (scan_kernel kPlane): the chunk-sum plane for one pooled
// directional track when the window reaches the neighbouring lanes only
static bool plane_scan(const up_ctx *c);
static int pool_mode(const up_ctx *c);
static bool pct_mode(const up_ctx *c);
static bool wide_mode(const up_ctx *c);

static bool want_index(const up_ctx *c);

int up_scan_density(up_ctx *c, uint32_t *b) {
    if (!c || !b) return UP_E_ARG;
    if (!c->have_params) return UP_E_STATE;
    // (the next pass: it builds the index first if it wants it)
    const bool plane = kTB == 2 && (c->p.bw + 64) / 64 <= 4 && want_index(c);
    *b = plane ? 1024u / 16u : 1024u * (uint32_t)kTB / 8u * (uint32_t)c->nc.size() * (c->p.nondir ? 2u : 1u);
    return UP_OK;
}

int up_set_index_policy(up_ctx *c, int policy) {
    if (!c || policy < UP_INDEX_AUTO || policy > UP_INDEX_ALWAYS) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // passes in flight read the unit table
    c->index_policy = policy;
    return UP_OK;
}

int up_invalidate_index(up_ctx *c) {
    if (!c) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;
    for (Unit &u : c->units) u.cs_dirty = u.pool_dirty = true;
    index_stale(c);
    return UP_OK;
}

int up_index_state(up_ctx *c, int *on, uint64_t *builds) {
    if (!c) return UP_E_ARG;
    if (on) *on = c->index_on ? 1 : 0;
    if (builds) *builds = c->index_builds;
    return UP_OK;
}

const char *up_strerror(int code) {
    switch (code) {
    case UP_OK: return "ok";
    case UP_E_ARG: return "bad argument";
    case UP_E_HIP: return "HIP runtime error";
    case UP_E_NOMEM: return "device memory exhausted";
    case UP_E_STATE: return "call out of order";
    case UP_E_UNSUPPORTED: return "configuration outside the GPU path";
    case UP_E_NODEV: return "no HIP device";
    case UP_E_INTERNAL: return "internal consistency check failed";
    default: return "unknown error";
    }
}

int up_device_count(int *n) {
    if (!n) return UP_E_ARG;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return UP_OK;
}

// Kernel::Kernel (misc/kernel.cpp:16-35): f(i/bw) = 3(1 - (i/bw)^2)/4 for
// i = -bw..bw, summed left to right, then every weight scaled by sum/total.
int up_kernel_weights(uint16_t bw, double sum, double *w) {
    if (!w) return UP_E_ARG;
    double acc = 0;
    for (int i = -(int)bw, j = 0; i <= (int)bw; ++i, ++j) {
        const double x = (double)i / (double)bw;
        const double x2 = x * x;
        w[j] = 3 * (1 - x2) / 4;
        acc += w[j];
    }
    const double scale = sum / acc;
    for (int j = 0; j < 2 * (int)bw + 1; ++j) w[j] *= scale;
    return UP_OK;
}

int up_open(int hip_device, up_ctx **out) {
    if (!out) return UP_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return UP_E_NODEV;
    if (hip_device < 0 || hip_device >= n) return UP_E_ARG;
    up_ctx *c = new up_ctx();
    c->dev = hip_device;
    HIPCHK(hipSetDevice(hip_device));
    HIPCHK(hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, hip_device));
    if (const char *e = getenv("UNIPEAK_K1A_PER_CU")) c->k1a_per_cu = atoi(e);
    if (const char *e = getenv("UNIPEAK_GRAPHS")) c->use_graphs = e[0] != '0';
    if (const char *e = getenv("UNIPEAK_K1B_PER_CU")) c->k1b_per_cu = atoi(e);
    if (const char *e = getenv("UNIPEAK_K3_PER_CU")) c->k3_per_cu = atoi(e);
    if (const char *e = getenv("UNIPEAK_K3_ONE")) c->k3_one = atoi(e) != 0;
    if (const char *e = getenv("UNIPEAK_CHAINS")) c->n_chain = std::min(4, std::max(1, atoi(e)));
    if (const char *e = getenv("UNIPEAK_LAUNCHER")) c->use_launcher = e[0] != '0';
    {
        int least = 0, greatest = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        // the context stream (track writes, the K0 head replays between
        // pipelined passes) at high priority: K0's few latency-bound waves
        // are dispatched ahead of the in-flight passes' queued K1b/K3 blocks
        // (configs[4], same box, three alternating pairs: 1.52-1.63 vs
        // 1.65-1.67 ms/step, profiles/r05/ctx_prio.txt); UNIPEAK_CTX_PRIO=0:
        // normal priority
        const char *ep = getenv("UNIPEAK_CTX_PRIO");
        HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking,
                                           (ep && ep[0] == '0') ? least : greatest));
        const char *e = getenv("UNIPEAK_K1A_PRIO");  // A/B: 0 = normal priority
        HIPCHK(hipStreamCreateWithPriority(&c->k1a_stream, hipStreamNonBlocking,
                                           (e && e[0] == '0') ? least : greatest));
        for (int i = 0; i < c->n_chain; ++i) HIPCHK(hipStreamCreateWithFlags(&c->chain[i], hipStreamNonBlocking));
    }
    for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
    for (auto &ps : c->pass) {
        for (auto &e : ps.ev) HIPCHK(hipEventCreate(&e));
        HIPCHK(hipEventCreateWithFlags(&ps.done, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ps.k1a_end, hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&c->host_work, hipEventDisableTiming));
    for (auto &e : c->scat_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = c;
    return UP_OK;
}

static void free_units(up_ctx *c) {
    for (auto &u : c->units) {
        if (u.dptr) (void)hipFree(u.dptr);
        if (u.d_ovf) (void)hipFree(u.d_ovf);
        if (u.d_ovf_off) (void)hipFree(u.d_ovf_off);
        if (u.d_ovf_tidx) (void)hipFree(u.d_ovf_tidx);
        if (u.d_ovf_tiles) (void)hipFree(u.d_ovf_tiles);
        if (u.d_pct) (void)hipFree(u.d_pct);
    }
    c->units.clear();
    c->units_dirty = true;
    c->ran = false;
}

static void drop_target(up_ctx *c);

static void launcher_stop(up_ctx *c);

void up_close(up_ctx *c) {
    if (!c) return;
    launcher_stop(c);
    (void)hipSetDevice(c->dev);
    (void)hipStreamSynchronize(c->stream);
    sync_all(c);
    free_units(c);
    drop_target(c);
    for (void *h : c->host_regs) (void)hipHostUnregister(h);
    c->d_kern.release(); c->d_coef.release(); c->d_nc.release(); c->d_ctl.release();
    c->d_units.release(); c->d_unit_last.release();
    c->d_resync.release(); c->d_emu_n.release(); c->d_emu_err.release();
    c->d_emu_counts.release(); c->d_ring_hits.release(); c->d_reg_hit.release(); c->d_reg_hits.release();
    c->d_unit_buffer.release(); c->d_reg_f.release(); c->d_reg_r.release(); c->d_emu_out.release();
    c->d_ring_f.release(); c->d_ring_r.release(); c->d_ring_has.release();
    c->d_emu_scores.release(); c->d_emu_score_off.release(); c->d_emu_nscores.release();
    c->d_sh_idx.release(); c->d_sh_off.release(); c->d_sh_slab.release(); c->d_sh_out.release();
    c->d_sh_pref.release();
    c->d_pf_unit.release(); c->d_pf_event.release(); c->d_pf_pos.release(); c->d_pf_score.release();
    c->d_pf_n.release();
    c->d_gunits.release(); c->d_goff.release(); c->d_gskip.release(); c->d_gstop.release();
    c->d_emu_group.release(); c->d_q11_head.release();
    c->d_seg.release(); c->d_seg_n.release(); c->d_gbeg.release(); c->d_gend.release();
    c->d_q11_stage.release(); c->d_q11_stage_cnt.release(); c->d_q11_tab.release(); c->d_q11_scr.release();
    c->d_q11_edit.release(); c->d_q11_st.release(); c->d_q11_en.release(); c->d_q11_src.release();
    for (int k = 0; k < kSlots; ++k) {
        c->hp_regions[k].release(); c->hp_counts[k].release(); c->hp_status[k].release(); c->hp_head[k].release();
        for (auto &e : c->pass[k].ev) (void)hipEventDestroy(e);
        (void)hipEventDestroy(c->pass[k].done);
        (void)hipEventDestroy(c->pass[k].k1a_end);
        for (auto &g : c->pass[k].graphs) (void)hipGraphExecDestroy(g.second);
        c->pass[k].release();
    }
    (void)hipStreamDestroy(c->k1a_stream);
    for (auto st : c->chain)
        if (st) (void)hipStreamDestroy(st);
    (void)hipEventDestroy(c->host_work);
    for (auto &e : c->scat_ev) (void)hipEventSynchronize(e);
    c->hp_scat[0].release(); c->hp_scat[1].release();
    for (auto &e : c->scat_ev) (void)hipEventDestroy(e);
    c->d_wscreen.release(); c->d_stage.release(); c->d_dbg.release(); c->d_pack_ovf.release(); c->d_pack_n.release();
    for (auto &e : c->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

static void set_q_params(up_ctx *c);

int up_set_params(up_ctx *c, const up_params *p) {
    if (!c || !p) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (p->n_samples == 0 || p->bw == 0) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    const int S = p->n_samples;
    std::vector<uint8_t> ctl(S, 0);
    if (p->is_control)
        for (int s = 0; s < S; ++s) ctl[s] = p->is_control[s] ? 1 : 0;
    std::vector<int32_t> nc;
    for (int s = 0; s < S; ++s)
        if (!ctl[s]) nc.push_back(s);
    std::vector<double> coef;
    if (p->n_coeffs) {
        if (!p->coeffs || p->n_coeffs != nc.size()) return UP_E_ARG;
        coef.assign(p->coeffs, p->coeffs + p->n_coeffs);
    }
    std::vector<double> kern(2 * p->bw + 1, 0.0);
    up_kernel_weights(p->bw, 1 / p->background, kern.data());
    // upload only what changed (a bench step re-sets identical parameters)
    const bool same = c->have_params && ctl == c->ctl && nc == c->nc && coef == c->coef &&
                      kern.size() == c->kern.size() &&
                      std::memcmp(kern.data(), c->kern.data(), kern.size() * sizeof(double)) == 0;
    const int old_bw = c->have_params ? c->p.bw : -1;
    c->p = *p;
    c->p.is_control = nullptr;
    c->p.coeffs = nullptr;
    if (!same) {
        c->ctl = ctl;
        c->nc = nc;
        c->coef = coef;
        c->kern = kern;
        HIPCHK(c->d_kern.ensure(c->kern.size()));
        HIPCHK(hipMemcpy(c->d_kern.p, c->kern.data(), c->kern.size() * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(c->d_nc.ensure(c->nc.size() + 1));
        if (!c->nc.empty())
            HIPCHK(hipMemcpy(c->d_nc.p, c->nc.data(), c->nc.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(c->d_ctl.ensure(S));
        HIPCHK(hipMemcpy(c->d_ctl.p, c->ctl.data(), S, hipMemcpyHostToDevice));
        // without coefficients: zeros, so the FP64 pooling (POOL 2) of
        // pool_mode's fallback sums 0 * c + c = c (the reference's countSum)
        std::vector<double> dc = c->coef.empty() ? std::vector<double>(c->nc.size() + 1, 0.0) : c->coef;
        HIPCHK(c->d_coef.ensure(dc.size() + 1));
        HIPCHK(hipMemcpy(c->d_coef.p, dc.data(), dc.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    // K1 screen: integer weight per non-control sample bounding its share of
    // |countSum| (1, or ceil(|coef| + 1) with coefficients, quirk Q5), and the
    // largest weighted window tag sum W with W * kmax * (1 + 1e-6) < thr
    {
        std::vector<uint32_t> w(c->nc.size() + 1, 1u);
        bool huge = false;
        for (size_t k = 0; k < c->coef.size(); ++k) {
            const double q = std::ceil(std::fabs(c->coef[k]) + 1.0);
            if (!(q <= 4096.0)) huge = true;
            w[k] = huge ? 1u : (uint32_t)q;
        }
        HIPCHK(c->d_wscreen.ensure(w.size()));
        HIPCHK(hipMemcpy(c->d_wscreen.p, w.data(), w.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        // the pooled planes follow the pooling (samples and their weights)
        std::vector<uint32_t> sig(c->nc.begin(), c->nc.end());
        sig.insert(sig.end(), w.begin(), w.end());
        if (sig != c->pool_sig) {
            c->pool_sig = sig;
            for (Unit &u : c->units) u.pool_dirty = true;
            c->units_dirty = true;
            index_stale(c);
        }
        double kmax = 0.0;
        for (double v : c->kern) kmax = v > kmax ? v : kmax;
        const double wf = p->region_thr / (kmax * (1.0 + 1e-6));
        uint32_t ws = 0;
        if (huge || !(wf > 0.0)) ws = 0;                    // screen off: any tag -> exact
        else if (wf >= (double)(kBig - 1)) ws = kBig - 1;
        else ws = (uint32_t)std::ceil(wf) - 1u;
        c->wskip = ws;
        // fine screen: fw[d] bounds the kernel weight between any two
        // positions of chunks d apart (smallest distance 0, 1, 17, 33, ...),
        // inflated by 1e-4; a chunk can hold a flag only if its bound > fthr
        const int bwi = p->bw;
        for (int d = 0; d <= kScrHalo; ++d) {
            const int u0 = d == 0 ? 0 : 16 * (d - 1) + 1;
            double kd = 0.0;
            for (int u = u0; u <= bwi; ++u) kd = std::max(kd, std::fabs(c->kern[bwi + u]));
            float f = (float)(kd * (1.0 + 1e-4));
            if ((double)f < kd * (1.0 + 1e-4)) f = std::nextafter(f, HUGE_VALF);
            c->fw[d] = f;
        }
        // screen off (huge coefficients): every tag within reach goes exact
        c->fthr = (huge || !(wf > 0.0)) ? 0.f : (float)(p->region_thr * (1.0 - 1e-6));
    }
    set_q_params(c);
    c->have_params = true;
    if (old_bw != p->bw) c->units_dirty = true;
    return UP_OK;
}

// K1b keys.  Kernel::Kernel (kernel.cpp:12-35) builds w_d = 3(1 - (d/bw)^2)/4
// times a scale, so the FP64 weight K_d = alpha (bw^2 - d^2) (1 + e_d) with
// alpha = K_0 / bw^2 and |e_d| <= E, measured here in long double (a few
// ulp for |d| << bw, up to ~bw/2 ulp next to the window edge where
// 1 - (d/bw)^2 cancels).  An FP64 score is a sum of <= 2bw+1 non-negative
// rounded products, added in some order, (+ the f + r add): within
// (2bw+3) ulp of its real value.  So score = alpha Q (1 +- delta) with
// delta = 2 (E + (2bw+4) 2^-53) (a factor 2 to spare).  The edge weights
// K_{+-bw} must be exactly 0 (they are: 1 - 1 = 0).
static void set_q_params(up_ctx *c) {
    c->q_ok = false;
    const int bw = c->p.bw;
    if (bw < 1 || bw > kMaxBw || (int)c->kern.size() != 2 * bw + 1 || !(c->p.region_thr > 0)) return;
    const long double b2 = (long double)bw * bw;
    const double k0 = c->kern[bw];
    if (!(k0 > 0) || c->kern[0] != 0.0 || c->kern[2 * bw] != 0.0) return;
    const double alpha = k0 / (double)(bw * bw);
    long double E = 0;
    for (int d = -bw + 1; d <= bw - 1; ++d) {
        const long double ideal = (long double)alpha * (b2 - (long double)d * d);
        const long double e = fabsl((long double)c->kern[bw + d] / ideal - 1.0L);
        if (!(e < 1e-9L)) return;  // not this kernel's shape
        E = e > E ? e : E;
    }
    const double delta = 2.0 * ((double)E + (2.0 * bw + 4.0) * 0x1p-53);
    // decided: Q <= qno -> alpha Q (1 + delta) < thr; Q >= qyes -> alpha Q (1 - delta) >= thr
    const double thr = c->p.region_thr;
    const double lo = thr / (alpha * (1.0 + delta)) * (1.0 - 1e-12) - 1.0;
    const double hi = thr / (alpha * (1.0 - delta)) * (1.0 + 1e-12) + 1.0;
    if (!(hi < 4294967295.0)) return;
    c->qno = lo < 0 ? 0u : (uint32_t)std::floor(lo);
    c->qyes = (uint32_t)std::ceil(hi);
    if (c->qyes < 1) c->qyes = 1;
    c->q_alpha = alpha;
    c->q_delta = delta;
    c->q_ok = true;
}

// Q keys for this pass: integer pooled counts (no -z coefficients), Q below
// 2^32 for the largest possible window, and distinct Q ordering the FP64
// scores: alpha (Q+1)(1 - delta) > alpha Q (1 + delta) for every Q <= Qmax
static bool q_mode(const up_ctx *c) {
    if (!c->q_ok || !c->coef.empty() || c->nc.empty() || c->p.bw > kMaxBw) return false;
    // several pooled samples: K3 would score each peak from every sample's
    // window bytes, which cost more than the keys save in K1b (hg19, 8
    // samples + 1 control: K1b 2.07 -> 1.64 ms but K3 0.82 -> 1.08-1.23 ms,
    // 541 -> 515-525 Gbp/s) -- unless K3 runs its own KDE anyway (-D with
    // the strand correlation), where the keys are K1b's gain only
    // (round 5, with the pooled count track, UNIPEAK_Q_POOLED=1: K3 scores
    // the pooled peak from one byte per window position, but configs[3]
    // still lost -- K1b 1.16 -> 1.13 ms, K3 0.54 -> 1.03 ms, 1,828 -> 1,458
    // Gbp/s same box, profiles/r05/pct/ -- so the keys stay off)
    const bool k3_kde = c->p.nondir && (c->p.want_corr || c->p.corr_thr > -1);
    static const bool q_pooled = [] {
        const char *e = getenv("UNIPEAK_Q_POOLED");
        return e && *e == '1';
    }();
    if (c->nc.size() > 1 && !k3_kde && !(q_pooled && pct_mode(c))) return false;
    const int bw = c->p.bw;
    const double cmax = (double)std::max<uint32_t>(kEsc - 1, c->ovf_max_all) * (double)c->nc.size() *
                        (c->p.nondir ? 2.0 : 1.0);
    const double qmax = (double)bw * bw * (2.0 * bw + 1.0) * cmax;
    return qmax < 4294967295.0 && 2.0 * c->q_delta * (qmax + 1.0) < 0.5;
}

// track geometry (bytes): positions 1..len plus the scan domain up to
// len+bw (Q16), rounded to whole strips, two positions per byte, with
// kPadBytes zero bytes on both sides
static uint64_t unit_stride(uint32_t len, int bw) {
    // (the scan domain [1, len + bw] and the windows around it, whose loads
    // reach len + 2bw; at least K1's widest kernel, kMaxBw; a later wider
    // -b regrows the unit, sync_layout)
    const uint64_t w = (uint64_t)std::max(bw, kMaxBw);
    const uint64_t dom = (uint64_t)len + 2 * w + 2;
    const uint64_t strips = (dom + kStrip - 1) / kStrip;
    return (uint64_t)kPadBytes + strips * kStripBytes + kPadBytes;
}

int up_add_unit(up_ctx *c, uint32_t len, int32_t nstrands, int32_t buffer_id, uint32_t *unit_id) {
    if (!c || !c->have_params || (nstrands != 1 && nstrands != 2)) return c && !c->have_params ? UP_E_STATE : UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (nstrands != (c->p.nondir ? 2 : 1)) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    Unit u;
    u.len = len;
    u.nstrands = nstrands;
    u.buffer = buffer_id;
    u.stride = unit_stride(len, c->p.bw);
    u.pad_bw = std::max<uint32_t>(c->p.bw, kMaxBw);
    // the tracks, their chunk-sum planes (stride / 4 bytes each, kernels.h),
    // the unit's pooled plane
    const size_t bytes = u.stride * (size_t)c->p.n_samples * nstrands / 4 * 5 + u.stride / 4;
    u.ovf.resize((size_t)c->p.n_samples * nstrands);
    hipError_t e = hipMalloc(&u.dptr, bytes);
    if (e != hipSuccess) return UP_E_NOMEM;
    HIPCHK(hipMemsetAsync(u.dptr, 0, bytes, c->stream));
    c->units.push_back(u);
    c->units_dirty = true;
    c->ran = false;
    if (unit_id) *unit_id = (uint32_t)(c->units.size() - 1);
    return UP_OK;
}

int up_unit_count(up_ctx *c, uint32_t *n) {
    if (!c || !n) return UP_E_ARG;
    *n = (uint32_t)c->units.size();
    return UP_OK;
}

int up_reset_units(up_ctx *c) {
    if (!c) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    (void)hipSetDevice(c->dev);
    (void)hipStreamSynchronize(c->stream);
    free_units(c);
    return UP_OK;
}

static uint8_t *track_ptr(up_ctx *c, uint32_t unit, int strand, uint16_t sample) {
    const Unit &u = c->units[unit];
    return u.dptr + ((uint64_t)strand * c->p.n_samples + sample) * u.stride;
}

static int check_track(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample) {
    if (!c || !c->have_params) return UP_E_STATE;
    if (unit >= c->units.size() || strand < 0 || strand >= c->units[unit].nstrands ||
        sample >= c->p.n_samples)
        return UP_E_ARG;
    return UP_OK;
}

// dense device uint32 counts -> the track (4-bit + overflow table)
static int pack_track(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, const uint32_t *src) {
    Unit &u = c->units[unit];
    const uint64_t len = u.len;
    if (len == 0) return UP_OK;
    HIPCHK(c->d_pack_n.ensure(1));
    uint32_t cap = (uint32_t)std::max<size_t>(c->d_pack_ovf.n, 4096);
    for (int attempt = 0; attempt < 2; ++attempt) {
        HIPCHK(c->d_pack_ovf.ensure(cap));
        HIPCHK(hipMemsetAsync(c->d_pack_n.p, 0, 4, c->stream));
        const uint64_t groups = (len + 4 * kPerByte - 1) / (4 * kPerByte);  // one dword per thread
        hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, c->stream,
                           track_ptr(c, unit, strand, sample), src, len, c->d_pack_ovf.p, c->d_pack_n.p, cap);
        HIPCHK(hipGetLastError());
        uint32_t n = 0;
        HIPCHK(hipMemcpyAsync(&n, c->d_pack_n.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (n > cap) { cap = n + n / 4; continue; }
        auto &m = u.ovf[(size_t)strand * c->p.n_samples + sample];
        m.clear();
        if (n) {
            std::vector<unsigned long long> e(n);
            HIPCHK(hipMemcpy(e.data(), c->d_pack_ovf.p, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            for (auto v : e) m[(uint32_t)(v >> 32)] = (uint32_t)v;
        }
        u.ovf_dirty = true;
        u.cs_dirty = u.pool_dirty = true;
        c->units_dirty = true;
        index_stale(c);
        return UP_OK;
    }
    return UP_E_INTERNAL;
}

int up_unit_pack(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, const uint32_t *dev_counts) {
    int r = check_track(c, unit, strand, sample);
    if (r) return r;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (!dev_counts) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    if ((r = pack_track(c, unit, strand, sample, dev_counts))) return r;
    c->ran = false;
    return UP_OK;
}

int up_unit_scatter(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, size_t n,
                    const uint32_t *pos, const uint32_t *counts) {
    int r = check_track(c, unit, strand, sample);
    if (r) return r;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (n == 0) return UP_OK;
    if (!pos || !counts) return UP_E_ARG;
    const uint32_t len = c->units[unit].len;
    bool ascending = true;
    for (size_t i = 0; i < n; ++i) {
        if (pos[i] == 0 || pos[i] > len) return UP_E_ARG;
        if (i && pos[i] <= pos[i - 1]) ascending = false;
    }
    if (!ascending) {  // positions must be unique: a nibble written twice in
                       // one call would OR two counts together (4-bit tracks)
        std::vector<uint32_t> sp(pos, pos + n);
        std::sort(sp.begin(), sp.end());
        if (std::adjacent_find(sp.begin(), sp.end()) != sp.end()) return UP_E_ARG;
    }
    HIPCHK(hipSetDevice(c->dev));
    {   // escapes: the host map holds every count >= kEsc of the track
        Unit &u = c->units[unit];
        auto &m = u.ovf[(size_t)strand * c->p.n_samples + sample];
        for (size_t i = 0; i < n; ++i) {
            if (counts[i] >= kEsc) { m[pos[i]] = counts[i]; u.ovf_dirty = true; }
            else if (!m.empty() && m.erase(pos[i])) u.ovf_dirty = true;
        }
        u.cs_dirty = u.pool_dirty = true;  // the chunk sums change with any count
        c->units_dirty = true;
        index_stale(c);
    }
    // the caller's arrays are copied into the staging buffers before we
    // return, so they may be reused at once; the kernels stay stream-ordered
    constexpr size_t kChunk = (size_t)4 << 20;
    uint8_t *track = track_ptr(c, unit, strand, sample);
    for (size_t off = 0; off < n; off += kChunk) {
        const size_t m = std::min(kChunk, n - off);
        const int k = c->scat_i;
        c->scat_i ^= 1;
        HIPCHK(hipEventSynchronize(c->scat_ev[k]));
        HIPCHK(c->hp_scat[k].ensure(2 * kChunk));
        std::memcpy(c->hp_scat[k].p, pos + off, m * sizeof(uint32_t));
        std::memcpy(c->hp_scat[k].p + kChunk, counts + off, m * sizeof(uint32_t));
        hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream,
                           track, c->hp_scat[k].dev, c->hp_scat[k].dev + kChunk, (uint64_t)m);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->scat_ev[k], c->stream));
    }
    c->ran = false;
    return UP_OK;
}

// ---- synthetic input (DESIGN.md "Synthetic input"; oracle/orc_synth.c) ----
static uint64_t hmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int up_unit_synth(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, uint64_t seed,
                  uint32_t contig_index, int32_t synth_strand, int32_t nondir, int32_t with_peaks) {
    return up_unit_synth_offset(c, unit, strand, sample, seed, contig_index, synth_strand, nondir,
                                with_peaks, 0);
}

int up_unit_synth_offset(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, uint64_t seed,
                         uint32_t contig_index, int32_t synth_strand, int32_t nondir,
                         int32_t with_peaks, int32_t offset) {
    return up_unit_synth_ex(c, unit, strand, sample, seed, contig_index, synth_strand, nondir,
                            with_peaks, offset, 0);
}

// peak_seed != 0: replicate mode -- the peak centres come from
// peak_seed's keys, shared by every sample generated with it; each sample
// draws its own height (tags per peak) and a centre jitter of -20..+20 bp
// from its own seed, and its own tag offsets
int up_unit_synth_ex(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, uint64_t seed,
                     uint32_t contig_index, int32_t synth_strand, int32_t nondir,
                     int32_t with_peaks, int32_t offset, uint64_t peak_seed) {
    if (offset < -32768 || offset > 32767) return UP_E_ARG;  // a short, like -s
    int r = check_track(c, unit, strand, sample);
    if (r) return r;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    HIPCHK(hipSetDevice(c->dev));
    const uint32_t len = c->units[unit].len;
    const int bw = c->p.bw;
    const uint64_t skey = hmix(seed);
    const uint64_t ckey = hmix(skey ^ (uint64_t)(contig_index + 1));
    const uint64_t tkey = hmix(ckey ^ (uint64_t)(0x100 + synth_strand));
    const uint64_t pckey = peak_seed ? hmix(hmix(peak_seed) ^ (uint64_t)(contig_index + 1)) : ckey;
    const uint64_t pkey = hmix(pckey ^ (uint64_t)(0x200 + (nondir ? 0 : synth_strand)));
    const int64_t lo = 2 * (int64_t)bw + 2, hi = (int64_t)len - 2 * (int64_t)bw - 1;
    if (hi < lo) return UP_OK;
    SynthThr thr;
    {
        const double lambda = 0.002925;
        double pr = std::exp(-lambda), cdf = pr;
        for (int k = 0; k < 6; ++k) {
            thr.t[k] = cdf >= 1.0 ? ~0ull : (uint64_t)(cdf * 18446744073709551616.0);
            pr *= lambda / (double)(k + 1);
            cdf += pr;
        }
    }
    HIPCHK(c->d_stage.ensure((size_t)len + 4));
    uint32_t *trk = c->d_stage.p;  // dense uint32 staging, packed below
    HIPCHK(hipMemsetAsync(trk, 0, (size_t)len * sizeof(uint32_t), c->stream));
    const uint64_t npos = (uint64_t)(hi - lo + 1);
    // device scratch of this call, freed on every return path after the
    // stream has drained (an early HIPCHK return included)
    struct StreamScratch {
        hipStream_t s;
        void *p[2] = {nullptr, nullptr};
        ~StreamScratch() {
            if (p[0] || p[1]) (void)hipStreamSynchronize(s);
            for (void *q : p)
                if (q) (void)hipFree(q);
        }
    } scratch{c->stream};
    uint64_t tab[1024];
    if (!peak_seed) {
        hipLaunchKernelGGL(synth_bg_kernel, dim3((unsigned)((npos + 255) / 256)), dim3(256), 0,
                           c->stream, trk, tkey, lo, hi, thr, (int64_t)offset, (int64_t)len);
    } else {
        // replicate mode: chunked Poisson background (synth_bgc_kernel)
        const double mu = 0.002925 * 65536.0;
        double pr = std::exp(-mu), cdf = pr;
        for (int k = 0; k < 1024; ++k) {
            tab[k] = cdf >= 1.0 ? ~0ull : (uint64_t)(cdf * 18446744073709551616.0);
            pr *= mu / (double)(k + 1);
            cdf += pr;
        }
        HIPCHK(hipMalloc(&scratch.p[0], sizeof tab));
        const uint64_t *d_tab = (const uint64_t *)scratch.p[0];
        // stream-ordered, then waited for: the source is this stack frame
        HIPCHK(hipMemcpyAsync(scratch.p[0], tab, sizeof tab, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const uint32_t nch = (uint32_t)((npos + 65535) >> 16);
        hipLaunchKernelGGL(synth_bgc_kernel, dim3((nch + 255) / 256), dim3(256), 0, c->stream, trk,
                           tkey, lo, hi, d_tab, (int64_t)offset, (int64_t)len, nch);
    }
    HIPCHK(hipGetLastError());
    if (with_peaks) {
        std::vector<uint32_t> tags;
        uint32_t npk = len / 150000u;
        if (npk < 1) npk = 1;
        int64_t clo, chi;
        if (len >= 20001u) { clo = 10000; chi = (int64_t)len - 10000; }
        else { clo = 2 * (int64_t)bw + 200; chi = (int64_t)len - 2 * (int64_t)bw - 200; }
        const int64_t shift = (nondir && synth_strand == 1) ? 150 : 0;
        for (uint32_t j = 0; chi >= clo && j < npk; ++j) {
            const uint64_t h = hmix(pkey ^ hmix(0x7065616B00000000ull + j));
            int64_t centre = clo + (int64_t)(h % (uint64_t)(chi - clo + 1));
            uint32_t n = 20u + (uint32_t)(hmix(h) % 180u);
            // replicate mode: the shared hash also picks the peak's kind --
            // 0/1 an artifact on strand 0/1 only, 2 a spike (every tag of every
            // sample at the shared centre), 3 a weak peak (2..11 tags per sample), else normal
            const uint32_t kind = peak_seed ? (uint32_t)(h >> 56) & 15u : 4u;
            if (peak_seed) {
                const uint64_t hs = hmix(h ^ skey);
                n = 20u + (uint32_t)(hs % 180u);
                if (kind != 2) centre += (int64_t)((hs >> 32) % 41u) - 20;
                if (kind == 3) n = 2u + (uint32_t)(hs % 10u);
                if (kind <= 1 && (uint32_t)synth_strand != kind) n = 0;
            }
            for (uint32_t i = 0; i < n; ++i) {
                int64_t s = 0;
                const uint64_t b = hmix(tkey ^ h ^ hmix(0x74616700000000ull + i));
                for (int m = 0; m < 12; ++m) s += (int64_t)(hmix(b + (uint64_t)m) >> 32);
                const int64_t off = kind == 2 ? 0 : (60 * (s - 6 * 4294967296ll) + 2147483648ll) >> 32;
                const int64_t p = centre + shift + off;
                // generated on [lo, hi]; the -s offset then moves it, and the
                // wiggle reader's bounds drop what leaves [1, len]
                if (p >= lo && p <= hi && p + offset >= 1 && p + offset <= (int64_t)len)
                    tags.push_back((uint32_t)(p + offset));
            }
        }
        if (!tags.empty()) {
            HIPCHK(hipMalloc(&scratch.p[1], tags.size() * sizeof(uint32_t)));
            uint32_t *d = (uint32_t *)scratch.p[1];
            HIPCHK(hipMemcpyAsync(d, tags.data(), tags.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(synth_peak_kernel, dim3((unsigned)((tags.size() + 255) / 256)), dim3(256), 0,
                               c->stream, trk, d, (uint64_t)tags.size());
            HIPCHK(hipGetLastError());
        }
    }
    HIPCHK(hipStreamSynchronize(c->stream));  // the scratch tables are read by the kernels above
    if ((r = pack_track(c, unit, strand, sample, trk))) return r;
    c->ran = false;
    return UP_OK;
}

int up_unit_tag_total(up_ctx *c, uint32_t unit, int32_t strand, uint16_t sample, uint64_t *total) {
    int r = check_track(c, unit, strand, sample);
    if (r) return r;
    if (!total) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    unsigned long long *d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(unsigned long long)));
    HIPCHK(hipMemsetAsync(d, 0, sizeof(unsigned long long), c->stream));
    const Unit &u = c->units[unit];
    hipLaunchKernelGGL(track_sum_kernel, dim3(1024), dim3(256), 0, c->stream,
                       track_ptr(c, unit, strand, sample), (uint64_t)u.stride, d);
    HIPCHK(hipGetLastError());
    unsigned long long h = 0;
    HIPCHK(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    (void)hipFree(d);
    for (const auto &kv : u.ovf[(size_t)strand * c->p.n_samples + sample]) h += kv.second;
    *total = h;
    return UP_OK;
}

int up_unit_set_last_add(up_ctx *c, uint32_t unit, uint32_t last) {
    if (!c || unit >= c->units.size()) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    c->units[unit].last_override = last;
    c->units[unit].has_override = true;
    return UP_OK;
}

static int sync_units(up_ctx *c);

int up_unit_last_add(up_ctx *c, uint32_t unit, uint32_t *last) {
    if (!c || !last || unit >= c->units.size()) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (c->units[unit].has_override) { *last = c->units[unit].last_override; return UP_OK; }
    if (!c->have_params) return UP_E_STATE;
    HIPCHK(hipSetDevice(c->dev));
    int r = sync_units(c);
    if (r) return r;
    const uint32_t nu = (uint32_t)c->units.size();
    HIPCHK(c->d_unit_last.ensure(nu));
    HIPCHK(hipMemsetAsync(c->d_unit_last.p, 0, nu * sizeof(uint32_t), c->stream));
    hipLaunchKernelGGL(unit_last_kernel, dim3(std::max(1u, std::min(2048u, (c->nstrips + 3) / 4))), dim3(256), 0,
                       c->stream, c->d_units.p, nu, c->nstrips, (int)c->p.n_samples, (int)c->nc.size(),
                       c->d_nc.p, c->d_unit_last.p);
    HIPCHK(hipGetLastError());
    c->unit_last.resize(nu);
    HIPCHK(hipMemcpyAsync(c->unit_last.data(), c->d_unit_last.p, nu * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *last = c->unit_last[unit];
    return UP_OK;
}

// every pass in flight has been launched and has finished on the device
// (its completion is still the caller's up_run_wait)
static void settle_in_flight(up_ctx *c);

// track geometry of a unit after a bw change that its padding does not
// cover: a larger allocation, every track copied at the new stride (the
// padding past the domain reads zeros); the index is rebuilt
static int regrow_unit(up_ctx *c, Unit &u) {
    const int S = c->p.n_samples;
    const uint64_t stride = unit_stride(u.len, c->p.bw);
    const size_t bytes = stride * (size_t)S * u.nstrands / 4 * 5 + stride / 4;
    uint8_t *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return UP_E_NOMEM;
    HIPCHK(hipMemsetAsync(p, 0, bytes, c->stream));
    HIPCHK(hipMemcpy2DAsync(p, stride, u.dptr, u.stride, u.stride, (size_t)S * u.nstrands, hipMemcpyDeviceToDevice,
                            c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    (void)hipFree(u.dptr);
    u.dptr = p;
    u.stride = stride;
    u.pad_bw = std::max<uint32_t>(c->p.bw, kMaxBw);
    if (u.d_pct) (void)hipFree(u.d_pct);
    u.d_pct = nullptr;
    u.cs_dirty = u.pool_dirty = true;
    return UP_OK;
}

// the unit layout: strips, overflow tables, escape bitmap, the unit table
static int sync_layout(up_ctx *c) {
    if (!c->units_dirty && c->bw_layout == c->p.bw) return UP_OK;
    c->aligned_valid = false;
    for (Unit &u : c->units)
        if ((uint32_t)c->p.bw > u.pad_bw) {
            if (int r = regrow_unit(c, u)) return r;
            index_stale(c);
        }
    std::vector<UnitDesc> &d = c->h_units;
    d.assign(c->units.size(), UnitDesc{});
    uint32_t strip = 0;
    for (size_t i = 0; i < c->units.size(); ++i) {
        Unit &u = c->units[i];
        // strips only serve the parallel scan (bw <= kMaxBw; wider kernels replay)
        const uint64_t dom = (uint64_t)u.len + (uint32_t)c->p.bw;
        u.nstrips = (uint32_t)((dom + kStrip - 1) / kStrip);
        u.strip0 = strip;
        strip += u.nstrips;
        if (u.ovf_dirty) {
            if (u.d_ovf) (void)hipFree(u.d_ovf);
            if (u.d_ovf_off) (void)hipFree(u.d_ovf_off);
            if (u.d_ovf_tidx) (void)hipFree(u.d_ovf_tidx);
            if (u.d_ovf_tiles) (void)hipFree(u.d_ovf_tiles);
            u.d_ovf = nullptr;
            u.d_ovf_off = nullptr;
            u.d_ovf_tidx = nullptr;
            u.d_ovf_tiles = nullptr;
            // entries sorted by (track, position), indexed per kOvfBlk positions
            std::vector<uint64_t> e;
            u.ovf_max = 0;
            const uint32_t nb = ovf_nblk(u.len);
            std::vector<uint32_t> off(u.ovf.size() * (size_t)(nb + 1), 0);
            // escape tiles: every block holding an escape gets kOvfBlk bytes
            // of min(count, 255) (ovf_lookup)
            std::vector<uint32_t> tidx(u.ovf.size() * (size_t)nb, kNoTile);
            std::vector<uint8_t> tiles;
            for (size_t t = 0; t < u.ovf.size(); ++t) {
                uint32_t *o = off.data() + t * (size_t)(nb + 1);
                uint32_t b = 0;
                for (const auto &kv : u.ovf[t]) {
                    const uint32_t kb = (uint32_t)((kv.first - 1) >> kOvfBlkShift);  // positions are 1-based
                    while (b <= kb) o[b++] = (uint32_t)e.size();
                    e.push_back(((uint64_t)kv.first << 32) | kv.second);
                    u.ovf_max = std::max(u.ovf_max, kv.second);
                    uint32_t &ti = tidx[t * (size_t)nb + kb];
                    if (ti == kNoTile) {
                        ti = (uint32_t)(tiles.size() / kOvfBlk);
                        tiles.resize(tiles.size() + kOvfBlk, 0);
                    }
                    tiles[(size_t)ti * kOvfBlk + ((kv.first - 1) & (kOvfBlk - 1))] =
                        (uint8_t)std::min<uint32_t>(kv.second, 255u);
                }
                while (b <= nb) o[b++] = (uint32_t)e.size();
            }
            if (!e.empty()) {
                HIPCHK(hipMalloc(&u.d_ovf, e.size() * sizeof(uint64_t)));
                HIPCHK(hipMalloc(&u.d_ovf_off, off.size() * sizeof(uint32_t)));
                HIPCHK(hipMalloc(&u.d_ovf_tidx, tidx.size() * sizeof(uint32_t)));
                HIPCHK(hipMalloc(&u.d_ovf_tiles, tiles.size()));
                HIPCHK(hipMemcpy(u.d_ovf, e.data(), e.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(u.d_ovf_off, off.data(), off.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(u.d_ovf_tidx, tidx.data(), tidx.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(u.d_ovf_tiles, tiles.data(), tiles.size(), hipMemcpyHostToDevice));
            }
            u.ovf_dirty = false;
        }
        d[i] = UnitDesc{(uint64_t)(uintptr_t)u.dptr, u.stride, u.len, u.strip0, u.nstrips, u.nstrands,
                        (uint64_t)(uintptr_t)u.d_ovf, (uint64_t)(uintptr_t)u.d_ovf_off,
                        (uint64_t)(uintptr_t)u.d_ovf_tidx, (uint64_t)(uintptr_t)u.d_ovf_tiles, 0};
    }
    c->nstrips = strip;
    c->ovf_max_all = 0;
    for (const Unit &u : c->units) c->ovf_max_all = std::max(c->ovf_max_all, u.ovf_max);
    {
        // escape bitmap: bit (strip) of row (strand * S + sample) is set when
        // a block of the strip, or the block either side (the screen's halos,
        // <= kScrHalo chunks < kOvfBlk), holds an escaped field of that track
        // (a function of the overflow entries, i.e. of the packed tracks:
        // part of the track format, not of the index)
        const uint32_t S = (uint32_t)std::max<int32_t>(1, (int32_t)c->p.n_samples);
        const uint32_t nw = (strip + 31) / 32;
        std::vector<uint32_t> esc((size_t)2 * S * nw, 0u);
        auto set = [&](size_t row, uint32_t g) { esc[row * nw + (g >> 5)] |= 1u << (g & 31); };
        for (const Unit &u : c->units) {
            for (size_t t = 0; t < u.ovf.size() && t < (size_t)2 * S; ++t) {
                for (const auto &kv : u.ovf[t]) {
                    const uint32_t kb = (uint32_t)((kv.first - 1) >> kOvfBlkShift);
                    const uint32_t local = kb / kBlocks;
                    if (local >= u.nstrips) continue;  // past the scan domain (cannot happen)
                    set(t, u.strip0 + local);
                    if (kb % kBlocks == 0 && local > 0) set(t, u.strip0 + local - 1);
                    if (kb % kBlocks == kBlocks - 1 && local + 1 < u.nstrips) set(t, u.strip0 + local + 1);
                }
            }
        }
        HIPCHK(c->d_esc.ensure(std::max<size_t>(esc.size(), 1)));
        if (!esc.empty())
            HIPCHK(hipMemcpy(c->d_esc.p, esc.data(), esc.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        c->esc_nw = nw;
    }
    c->index_on = false;  // the table below carries no pooled count tracks
    HIPCHK(c->d_units.ensure(d.size()));
    if (!d.empty()) HIPCHK(hipMemcpy(c->d_units.p, d.data(), d.size() * sizeof(UnitDesc), hipMemcpyHostToDevice));
    c->units_dirty = false;
    c->bw_layout = c->p.bw;
    return UP_OK;
}

// Index policy: whether the next pass uses the per-dataset
// index -- chunk-sum planes, pooled planes, pooled count tracks, all derived
// from the packed tracks.  K1w screens on the planes, so it always does.
static bool want_index(const up_ctx *c) {
    if (kTB != 2) return false;
    if (wide_mode(c)) return true;
    switch (c->index_policy) {
    case UP_INDEX_ALWAYS: return true;
    case UP_INDEX_NEVER: return false;
    default: return c->passes_on_tracks >= 1;  // UP_INDEX_AUTO: from the second pass on
    }
}

// build what the index lacks (one launch per kind over every stale unit) and
// switch the unit table and the passes to it -- or off it
static int sync_index(up_ctx *c) {
    const bool want = want_index(c);
    const bool want_pct = pct_mode(c);
    const bool pooled = c->p.nondir || pool_mode(c) != 0;
    bool stale = false;
    for (const Unit &u : c->units)
        stale |= u.cs_dirty || (pooled && u.pool_dirty) || (want_pct && !u.d_pct) || (!want_pct && u.d_pct);
    if (want && stale) {
        if (busy(c)) settle_in_flight(c);  // (UP_INDEX_AUTO's second pass: the first one ran without it)
        const int S = c->p.n_samples;
        std::vector<uint32_t> lc, lp, lt;
        std::vector<uint64_t> oc{0}, op{0}, ot{0};
        std::vector<uint8_t *> pt;
        for (size_t i = 0; i < c->units.size(); ++i) {
            Unit &u = c->units[i];
            if (want_pct && !u.d_pct) {
                HIPCHK(hipMalloc(&u.d_pct, (size_t)u.nstrands * kPerByte * u.stride));
                u.pool_dirty = true;
            } else if (!want_pct && u.d_pct) {
                (void)hipFree(u.d_pct);
                u.d_pct = nullptr;
            }
            if (u.cs_dirty) {
                lc.push_back((uint32_t)i);
                oc.push_back(oc.back() + u.stride / 16 * (uint64_t)u.nstrands * S);
                u.pool_dirty = true;  // (the pooled plane sums the track planes)
            }
            if (pooled && u.pool_dirty) {
                lp.push_back((uint32_t)i);
                op.push_back(op.back() + u.stride / 16);
                if (u.d_pct) {
                    lt.push_back((uint32_t)i);
                    ot.push_back(ot.back() + u.stride / 4 * (uint64_t)u.nstrands);
                    pt.push_back(u.d_pct);
                }
            }
        }
        // one device block of lists: [lc | lp | lt] ids, their prefixes, pct pointers
        const size_t nid = lc.size() + lp.size() + lt.size(), noff = oc.size() + op.size() + ot.size();
        std::vector<uint64_t> blob(nid + noff + pt.size());
        uint32_t *ids = (uint32_t *)blob.data();  // (nid uint32s fit in nid uint64s)
        std::copy(lc.begin(), lc.end(), ids);
        std::copy(lp.begin(), lp.end(), ids + lc.size());
        std::copy(lt.begin(), lt.end(), ids + lc.size() + lp.size());
        uint64_t *offs = blob.data() + nid;
        std::copy(oc.begin(), oc.end(), offs);
        std::copy(op.begin(), op.end(), offs + oc.size());
        std::copy(ot.begin(), ot.end(), offs + oc.size() + op.size());
        for (size_t k = 0; k < pt.size(); ++k) blob[nid + noff + k] = (uint64_t)(uintptr_t)pt[k];
        HIPCHK(c->d_index_lists.ensure(std::max<size_t>(blob.size(), 1)));
        uint64_t *db = c->d_index_lists.p;
        HIPCHK(hipMemcpyAsync(db, blob.data(), blob.size() * 8, hipMemcpyHostToDevice, c->stream));
        const uint32_t *dids = (const uint32_t *)db;
        const uint64_t *doff = db + nid;
        auto grid = [](uint64_t items) { return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, 8192))); };
        if (!lc.empty())
            hipLaunchKernelGGL(csum_units_kernel, grid(oc.back()), dim3(256), 0, c->stream, c->d_units.p, dids, doff,
                               (uint32_t)lc.size(), S);
        if (!lp.empty())
            hipLaunchKernelGGL(pool_units_kernel, grid(op.back()), dim3(256), 0, c->stream, c->d_units.p,
                               dids + lc.size(), doff + oc.size(), (uint32_t)lp.size(), S, (int)c->nc.size(),
                               c->d_nc.p, c->d_wscreen.p);
        if (!lt.empty())
            hipLaunchKernelGGL(pct_units_kernel, grid(ot.back()), dim3(256), 0, c->stream, c->d_units.p,
                               dids + lc.size() + lp.size(), doff + oc.size() + op.size(), (uint32_t)lt.size(), S,
                               (int)c->nc.size(), c->d_nc.p, (uint8_t *const *)(db + nid + noff));
        HIPCHK(hipGetLastError());
        for (Unit &u : c->units) {
            u.cs_dirty = false;
            if (pooled) u.pool_dirty = false;
        }
        HIPCHK(hipStreamSynchronize(c->stream));  // (the host blob above is freed on return)
        ++c->index_builds;
        stale = false;
    }
    const bool on = want && !stale;
    if (on != c->index_on) {
        if (busy(c)) settle_in_flight(c);  // passes in flight read the unit table
        for (size_t i = 0; i < c->units.size(); ++i)
            c->h_units[i].pct = on ? (uint64_t)(uintptr_t)c->units[i].d_pct : 0;
        if (!c->h_units.empty())
            HIPCHK(hipMemcpy(c->d_units.p, c->h_units.data(), c->h_units.size() * sizeof(UnitDesc),
                             hipMemcpyHostToDevice));
        c->index_on = on;
    }
    return UP_OK;
}

static int sync_units(up_ctx *c) {
    if (int r = sync_layout(c)) return r;
    return sync_index(c);
}

// 0: one non-control sample; 1: several, summed in uint32 window words
// (kernels.hip WinT) -- only while no position's sum can reach 2^32, else
// 2 with zero coefficients (d_coef), the FP64 pooling of -z (quirk Q5)
static int pool_mode(const up_ctx *c) {
    if (!c->coef.empty()) return 2;
    if (c->nc.size() == 1) return 0;
    const double cmax = (double)std::max<uint32_t>(kEsc - 1, c->ovf_max_all) * (double)c->nc.size();
    return cmax < 4294967296.0 ? 1 : 2;
}

// pooled count tracks (UnitDesc::pct) for this pooling; UNIPEAK_PCT=0: off
// (every pooled sample's track, as before round 5)
static bool pct_mode(const up_ctx *c) {
    static const bool on = [] {
        const char *e = getenv("UNIPEAK_PCT");
        return !(e && *e == '0');
    }();
    return on && kTB == 2 && pool_mode(c) == 1;
}

static bool plane_scan(const up_ctx *c) {
    return kTB == 2 && (c->p.bw + 64) / 64 <= 4 && c->index_on;
}

static ScanParams scan_params(up_ctx *c, up_ctx::Pass &ps, uint32_t ovf_cap) {
    ScanParams P{};
    P.units = c->d_units.p;
    P.nunits = (uint32_t)c->units.size();
    P.nstrips = c->nstrips;
    P.S = c->p.n_samples;
    P.nnc = (int32_t)c->nc.size();
    P.nc = c->d_nc.p;
    P.coef = c->d_coef.p;
    P.kern = c->d_kern.p;
    P.wscreen = c->d_wscreen.p;
    P.wskip = c->wskip;
    for (int d = 0; d <= kScrHalo; ++d) P.fw[d] = c->fw[d];
    P.fthr = c->fthr;
    P.bw = c->p.bw;
    P.thr = c->p.region_thr;
    P.strip_info = ps.d_info.p;
    P.rec = ps.d_rec.p;
    P.ovf_count = ps.d_ovf_count.p;
    P.ovf_rec = ps.d_ovf_rec.p;
    P.ovf_cap = ovf_cap;
    P.xlist = ps.d_xlist.p;
    P.xwcount = ps.d_xwcount.p;
    P.xref = ps.d_xref.p;
    P.xcount = ps.d_xcount.p;
    P.spk = ps.d_spk.p;
    P.qmode = q_mode(c) ? 1 : 0;
    P.qno = c->qno;
    P.qyes = c->qyes;
    P.esc = c->esc_nw ? c->d_esc.p : nullptr;
    P.esc_nw = c->esc_nw;
    return P;
}

// Workgroups of `kernel` (256 threads, `lds` bytes of dynamic LDS) that are
// resident on the whole device at once.  The grid-stride kernels launch
// exactly this many: a larger grid leaves its last workgroups waiting for a
// slot and finishing their share of the work list after everyone else (a
// tail of up to one whole per-workgroup share).
static uint32_t resident_blocks(const up_ctx *c, const void *kernel, size_t lds, int threads = 256) {
    static std::mutex mu;
    static std::map<std::pair<const void *, size_t>, int> per_cu;
    int n = 0;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = per_cu.find({kernel, lds});
        if (it != per_cu.end()) {
            n = it->second;
        } else {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, lds) != hipSuccess || n < 1) n = 1;
            per_cu[{kernel, lds}] = n;
        }
    }
    return (uint32_t)n * (uint32_t)(c->ncu > 0 ? c->ncu : 256);
}

template <bool PROF, int MODE>
static void dispatch_scan(up_ctx *c, hipStream_t st, const ScanParams &P, uint32_t b, uint32_t e) {
    constexpr bool kScr = MODE == kModeScreen || MODE == kModeScreenF;
    const size_t lds = kScr ? kScreenLds : MODE == kModeExact ? kExactLds : kScanLds;
    const void *k = scan_kernel_for(P.bw, pool_mode(c), c->p.nondir != 0, PROF, MODE);
    uint32_t blocks = resident_blocks(c, k, lds);
    if (MODE == kModeExact) {
        // K1b: grid-stride over the device-side work-list count, the
        // resident grid.  Round 1 launched twice that (the 8-GPU plan's rank:
        // 57 vs 82 us with the FP64 walk); with the keys' cheaper items the
        // resident grid is as fast there and 2.8 % faster at N=1 (hg19, four
        // alternating pairs: 4,332 vs 4,214 Gbp/s, UNIPEAK_K1B_PER_CU A/B)
        if (c->k1b_per_cu > 0) blocks = (uint32_t)c->k1b_per_cu * (uint32_t)(c->ncu > 0 ? c->ncu : 256);
    } else {
        if (kScr) {
            // K1a leaves room on every CU for the previous pass's K1b/K3
            // (they overlap it, launch_pass): k1a_per_cu workgroups per CU
            const uint32_t cap = (uint32_t)c->k1a_per_cu * (uint32_t)(c->ncu > 0 ? c->ncu : 256);
            if (c->k1a_per_cu > 0 && cap < blocks) blocks = cap;
        }
        const uint32_t need = (e - b + 3) / 4;  // one wave per strip at most
        if (need < blocks) blocks = need;
        if (blocks > kMaxK1aWaves / 4) blocks = kMaxK1aWaves / 4;
        if (blocks == 0) return;
    }
    ScanParams Q = P;
    if (kScr) {  // per-wave work-list stash regions (ScanParams::xlist)
        c->k1a_waves = 4 * blocks;
        c->k1a_xcap = Q.xcap = (e - b + c->k1a_waves - 1) / c->k1a_waves;
    }
    void *args[] = {&Q, &b, &e};
    (void)hipLaunchKernel(k, dim3(blocks), dim3(256), args, lds, st);
}

static StatParams stat_params(up_ctx *c, up_ctx::Pass &ps) {
    StatParams P{};
    P.units = c->d_units.p;
    P.S = c->p.n_samples;
    P.nnc = (int32_t)c->nc.size();
    P.nc = c->d_nc.p;
    P.is_control = c->d_ctl.p;
    P.coef = c->d_coef.p;
    P.kern = c->d_kern.p;
    P.bw = c->p.bw;
    P.nondir = c->p.nondir;
    P.want_corr = c->p.want_corr || c->p.corr_thr > -1;
    P.region_thr = c->p.region_thr;
    P.kurt_thr = c->p.kurt_thr;
    P.corr_thr = c->p.corr_thr;
    P.hit_thr = c->p.hit_thr;
    P.starts = ps.d_starts.p;
    P.ends = ps.d_ends.p;
    P.reg_unit = ps.d_runit.p;
    P.peak_pos = nullptr;  // set by up_run (known peaks from K1)
    P.peak_val = nullptr;
    P.nreg = ps.d_nreg.p;
    P.out = nullptr;  // set by up_run (mapped host records)
    P.out_counts = nullptr;
    P.cap = 0;
    P.qmode = q_mode(c) ? 1 : 0;
    P.planes = c->index_on ? 1 : 0;
    static const int k3l_cut = [] {
        const char *e = getenv("UNIPEAK_K3L_CUT");
        return e && *e ? atoi(e) : 0;
    }();
    P.cut = k3l_cut;
    static const int k3l_heavy = [] {
        const char *e = getenv("UNIPEAK_K3L_HEAVY");
        return e && *e ? atoi(e) : kK3LHeavy;
    }();
    P.heavy = k3l_heavy;
    static const int k3l_w2 = [] {
        const char *e = getenv("UNIPEAK_K3L_W2");
        return e && *e ? atoi(e) : 1;
    }();
    P.w2hits = k3l_w2;
    return P;
}

static void dispatch_stats(up_ctx *c, hipStream_t st, const StatParams &P, uint64_t nreg) {
    // one pooled directional sample with K1b's peaks: the batched K3
    // (stats1.hip; UNIPEAK_K3_ONE=0 keeps the general kernel, for A/B and tests)
    const bool one = c->k3_one && kTB == 2 && pool_mode(c) == 0 && c->p.nondir == 0 && c->p.n_samples == 1 &&
                     P.peak_pos != nullptr;
    // one: a lane per region (stats1L_kernel, round 6; UNIPEAK_K3_LANE=0: a
    // wave per region, stats1_kernel)
    // (UNIPEAK_K3_LANE=2: a lane per region whatever the count, for A/B)
    static const int lane_k3 = [] {
        const char *e = getenv("UNIPEAK_K3_LANE");
        return e && *e ? atoi(e) : 1;
    }();
    // K3L's time is its slowest lane's region (escaped counts resolved one
    // by one at a large peak), whatever the region count: with many regions
    // its few waves leave the overlapping K1a/K1b more of the GPU (configs[1]
    // N = 1: 0.4304 / 0.4294 vs 0.4531 / 0.4356 ms per step), with the few of
    // an 8-GPU rank's shard (~5,200) the wave-per-region kernel finishes
    // sooner (simulated rank 4: 0.0779 / 0.0777 vs 0.1339 / 0.1322 ms;
    // profiles/r06/ab_k3.txt) -- the pass's estimate of its region count
    // (the last pass's) picks
    constexpr uint64_t kK3LaneMin = 16384;
    const int kind = one ? ((lane_k3 == 2 || (lane_k3 == 1 && nreg >= kK3LaneMin)) ? 2 : 1) : 0;
    // (beyond 256 samples one LDS row of exptSums per wave, kernels.hip add_es)
    const size_t lds = kind == 2 ? kStat1LLds : kind == 1 ? kStat1Lds
                                                          : kStatLds + (c->p.n_samples > 256 ? 4 * 4 * (size_t)c->p.n_samples : 0);
    const void *k = stats_kernel_for(P.bw, pool_mode(c), c->p.nondir != 0, kind);
    uint64_t cap = resident_blocks(c, k, lds, kind == 2 ? kK3LThreads : 256);
    if (c->k3_per_cu > 0) cap = std::min<uint64_t>(cap, (uint64_t)c->k3_per_cu * (uint64_t)(c->ncu > 0 ? c->ncu : 256));
    // (a lane per region: 256 regions per block; the kernels grid-stride past the estimate)
    const uint64_t blocks = std::min<uint64_t>(kind == 2 ? (nreg + kK3LThreads - 1) / kK3LThreads : (nreg + 3) / 4, cap);
    if (blocks == 0) return;
    StatParams Q = P;
    void *args[] = {&Q};
    (void)hipLaunchKernel(k, dim3((unsigned)blocks), dim3(kind == 2 ? kK3LThreads : 256), args, lds, st);
}

// Configurations the parallel scan does not represent run through the
// exact state machine over every unit (K0 replay, emulate.hip): a threshold
// <= 0 makes the leap branch of processPosition live (quirk Q11, the leap
// position joins a region without setting its left end), and kernels wider
// than kMaxBw exceed the scan's register-resident halo.
// A threshold <= 0 with non-negative scores (no negative coefficient) runs
// in parallel instead (K1q, run_q11): every processed position qualifies, so
// regions are the runs of processed positions; units that start processing
// at position 1 still take the replay.  UNIPEAK_Q11_REPLAY=1: always replay.
static bool q11_mode(const up_ctx *c) {
    if (c->p.region_thr > 0 || c->p.bw > kMaxBw || kTB != 2) return false;
    for (double q : c->coef)
        if (!(q >= 0)) return false;
    static const bool off = [] {
        const char *e = getenv("UNIPEAK_Q11_REPLAY");
        return e && *e && *e != '0';
    }();
    return !off;
}

// UNIPEAK_Q11_HEADS=replay: units that process position 1 send the whole
// context to the whole-buffer replay (round 4's rule; A/B and tests)
static bool q11_whole_replay() {
    static const bool on = [] {
        const char *e = getenv("UNIPEAK_Q11_HEADS");
        return e && std::strcmp(e, "replay") == 0;
    }();
    return on;
}

// K1w (wide.hip) for kernels wider than K1's halo: directional units, a
// threshold > 0, no -w capture (its retirements come from the replay), and
// a window of at most 65,535 cells (bw <= kMaxWideBw): the reference counts
// the cells add() retires in a UShort (misc/peakcall.cpp:172-177), so from
// bw 32,768 on a gap of 2bw + 1 or more retires (gap mod 65,536) cells, the
// rest of the window stays misaligned and a flush leaks into the buffer's
// next unit -- only the whole-buffer replay models that (emulate.hip);
// UNIPEAK_WIDE=0: the replay instead
static bool wide_mode(const up_ctx *c) {
    static const bool on = [] {
        const char *e = getenv("UNIPEAK_WIDE");
        return !(e && *e == '0');
    }();
    return on && c->p.bw > kMaxBw && c->p.bw <= kMaxWideBw && kTB == 2 && c->p.region_thr > 0 && !c->p.nondir &&
           !c->prof_capture;
}

static bool replay_mode(const up_ctx *c) {
    return (c->p.bw > kMaxBw && !wide_mode(c)) || (!(c->p.region_thr > 0) && !q11_mode(c));
}

static int check_params(up_ctx *c) {
    if (!c || !c->have_params) return UP_E_STATE;
    if (c->p.bw < 1) return UP_E_ARG;
    if (c->p.n_samples > kMaxSamples) return UP_E_UNSUPPORTED;
    return UP_OK;
}

// the parallel scan; K1q passes only inside the blocking up_run (their
// records are finished on the host), K1q's dense profile always
static int check_runnable(up_ctx *c, bool profile = false) {
    int r = check_params(c);
    if (r) return r;
    if (replay_mode(c)) return UP_E_UNSUPPORTED;
    if (profile && c->p.bw > kMaxBw) return UP_E_UNSUPPORTED;  // (the dense profile's window is K1's)
    return q11_mode(c) && !c->q11_run && !profile ? UP_E_UNSUPPORTED : UP_OK;
}

// Quirk Q1: units whose pooled hits include a position <= bw are replayed
// by the exact state machine (emulate.hip); their early regions replace the
// parallel path's, and the merged list moves to the host.
// K2a (segment counts of every strip) + quirk-Q1 head detection (units with
// pooled tags at positions <= bw, misc/peakcall.cpp:177-183) in one launch
static int launch_seg_count_head(up_ctx *c, int slot) {
    up_ctx::Pass &ps = c->pass[slot];
    const uint32_t nu = (uint32_t)c->units.size();
    const uint32_t ns = c->nstrips;
    const uint32_t nsb = (ns + kSegBlock - 1) / kSegBlock;
    HIPCHK(ps.d_head.ensure(nu));
    HIPCHK(c->hp_head[slot].ensure(nu));
    if (pool_mode(c) == 2)
        hipLaunchKernelGGL(seg_count_head_kernel<2>, dim3(nsb + nu), dim3(kSegBlock), 0, ps.stream, ps.d_info.p,
                           ps.d_cnt.p, ps.d_bsum.p, ns, nsb, c->d_units.p, (int)c->p.n_samples,
                           (int)c->nc.size(), c->d_nc.p, c->d_coef.p, (int)c->p.bw, ps.d_head.p,
                           c->hp_head[slot].dev);
    else
        hipLaunchKernelGGL(seg_count_head_kernel<1>, dim3(nsb + nu), dim3(kSegBlock), 0, ps.stream, ps.d_info.p,
                           ps.d_cnt.p, ps.d_bsum.p, ns, nsb, c->d_units.p, (int)c->p.n_samples,
                           (int)c->nc.size(), c->d_nc.p, c->d_coef.p, (int)c->p.bw, ps.d_head.p,
                           c->hp_head[slot].dev);
    HIPCHK(hipGetLastError());
    return UP_OK;
}

// threshold <= 0 chains for K0 (run_q11): group g = units gunits[goff[g] ..
// goff[g + 1]) of one buffer, replayed from position gskip[g] of its first
// unit; out: where each group stopped (unit, leap position; ~0: ran to its
// end) and the group of each replayed record
struct Q11Chains {
    std::vector<uint32_t> gunits, goff{0}, gskip;
    std::vector<uint32_t> gbeg, gend;  // instead of goff: ranges of gunits (segmented replay)
    std::vector<uint32_t> gstop, rgroup;
};

// K0: run the exact state machine (emulate.hip) over the units flagged in
// d_head (replay_all: over every unit, never resynced; q: the threshold <= 0
// chains instead) -> its regions, their exptSums and the per-unit resync
// positions.  Capacity of the region record area and of one open region
// grow until the replay fits.
static int emulate_units(up_ctx *c, const uint32_t *d_head, bool replay_all, std::vector<up_region> &emu,
                         std::vector<uint32_t> &ecnt,
                         std::vector<uint32_t> &resync, std::vector<uint64_t> &soff, Q11Chains *q = nullptr) {
    const uint32_t nu = (uint32_t)c->units.size();
    const int S = c->p.n_samples;
    const uint32_t W = 2u * c->p.bw + 1;
    std::vector<int32_t> ub(nu);
    for (uint32_t i = 0; i < nu; ++i) ub[i] = c->units[i].buffer;
    HIPCHK(c->d_unit_buffer.ensure(nu));
    HIPCHK(hipMemcpy(c->d_unit_buffer.p, ub.data(), nu * sizeof(int32_t), hipMemcpyHostToDevice));
    // chain groups (EmuParams::gunits): the whole buffer when every unit is
    // replayed; otherwise a new group after every unit with an add past bw
    // (it cannot leave state behind), so independent head-hit units replay in
    // parallel instead of one wave walking the buffer
    std::vector<uint32_t> aligned(nu, 0);
    if (!replay_all && !q && nu && c->aligned_valid && c->aligned_cache.size() == nu) {
        aligned = c->aligned_cache;  // (a function of the tracks and bw: once per layout)
    } else if (!replay_all && !q && nu) {
        HIPCHK(c->d_q11_head.ensure(nu));
        HIPCHK(hipMemsetAsync(c->d_q11_head.p, 0, nu * sizeof(uint32_t), c->stream));
        hipLaunchKernelGGL(unit_aligned_kernel, dim3(nu), dim3(256), 0, c->stream, c->d_units.p, S, (int)c->p.bw,
                           c->d_q11_head.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(aligned.data(), c->d_q11_head.p, nu * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->aligned_cache = aligned;
        c->aligned_valid = true;
    }
    std::vector<std::vector<uint32_t>> groups;
    {
        int64_t open[2] = {-1, -1};  // the buffer's current group
        for (uint32_t u = 0; u < nu; ++u) {
            const int b = c->units[u].buffer;
            if (open[b] < 0) {
                open[b] = (int64_t)groups.size();
                groups.emplace_back();
            }
            groups[open[b]].push_back(u);
            if (!replay_all && aligned[u]) open[b] = -1;
        }
    }
    std::vector<uint32_t> gunits, goff{0};
    if (q) {
        gunits = q->gunits;
        goff = q->goff;
    } else {
        for (const auto &g : groups) {
            gunits.insert(gunits.end(), g.begin(), g.end());
            goff.push_back((uint32_t)gunits.size());
        }
    }
    const bool ranges = q && !q->gbeg.empty();
    const uint32_t ngroups = ranges ? (uint32_t)q->gbeg.size() : (uint32_t)goff.size() - 1;
    HIPCHK(c->d_gunits.ensure(std::max<size_t>(gunits.size(), 1)));
    HIPCHK(c->d_goff.ensure(goff.size()));
    if (!gunits.empty())
        HIPCHK(hipMemcpy(c->d_gunits.p, gunits.data(), gunits.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_goff.p, goff.data(), goff.size() * 4, hipMemcpyHostToDevice));
    if (q) {
        if (q->gskip.size() != ngroups) return UP_E_INTERNAL;
        if (ranges) {
            HIPCHK(c->d_gbeg.ensure(ngroups));
            HIPCHK(c->d_gend.ensure(ngroups));
            HIPCHK(hipMemcpy(c->d_gbeg.p, q->gbeg.data(), ngroups * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->d_gend.p, q->gend.data(), ngroups * 4, hipMemcpyHostToDevice));
        }
        HIPCHK(c->d_gskip.ensure(std::max(ngroups, 1u)));
        HIPCHK(c->d_gstop.ensure(2 * std::max(ngroups, 1u)));
        if (ngroups) HIPCHK(hipMemcpy(c->d_gskip.p, q->gskip.data(), ngroups * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(c->d_resync.ensure(nu));
    HIPCHK(c->d_emu_n.ensure(1));
    HIPCHK(c->d_emu_err.ensure(1));
    // the window in LDS when it fits (64 KiB), else in global scratch
    const size_t ring_bytes = (size_t)W * (2 * sizeof(double) + 1);
    const bool ring_lds = ring_bytes + sizeof(EmuLds) <= 65536 - 64;
    for (int attempt = 0;; ++attempt) {
        if (attempt == 6) return UP_E_NOMEM;
        uint32_t &reg_cap_ref = q ? c->emu_chain_reg_cap : c->emu_reg_cap;
        const uint32_t reg_cap = reg_cap_ref, out_cap = c->emu_out_cap;
        // workgroups (scratch slots): every group at once, within ~1 GiB of scratch
        const uint64_t slot_bytes = (uint64_t)W * S * 4 + (uint64_t)reg_cap * (8 + 8 + 4 + 4ull * S) +
                                    (ring_lds ? 0 : (uint64_t)W * 17);
        const uint32_t nslots = (uint32_t)std::max<uint64_t>(
            1, std::min<uint64_t>({(uint64_t)std::max(ngroups, 1u), q ? 2048u : 256u,
                                   (1ull << 30) / std::max<uint64_t>(slot_bytes, 1)}));
        HIPCHK(c->d_ring_hits.ensure((uint64_t)nslots * W * S));
        if (!ring_lds) {
            HIPCHK(c->d_ring_f.ensure((uint64_t)nslots * W));
            HIPCHK(c->d_ring_r.ensure((uint64_t)nslots * W));
            HIPCHK(c->d_ring_has.ensure((uint64_t)nslots * W));
        }
        HIPCHK(hipMemsetAsync(c->d_resync.p, 0, nu * sizeof(uint32_t), c->stream));
        HIPCHK(hipMemsetAsync(c->d_emu_n.p, 0, 4, c->stream));
        HIPCHK(hipMemsetAsync(c->d_emu_err.p, 0, 4, c->stream));
        HIPCHK(c->d_emu_nscores.ensure(1));
        HIPCHK(hipMemsetAsync(c->d_emu_nscores.p, 0, sizeof(unsigned long long), c->stream));
        HIPCHK(c->d_emu_scores.ensure(c->emu_scores_cap));
        HIPCHK(c->d_emu_score_off.ensure(out_cap));
        if (!ring_lds) {
            HIPCHK(hipMemsetAsync(c->d_ring_f.p, 0, (uint64_t)nslots * W * sizeof(double), c->stream));
            HIPCHK(hipMemsetAsync(c->d_ring_r.p, 0, (uint64_t)nslots * W * sizeof(double), c->stream));
            HIPCHK(hipMemsetAsync(c->d_ring_has.p, 0, (uint64_t)nslots * W, c->stream));
        }
        HIPCHK(c->d_emu_out.ensure(out_cap));
        HIPCHK(c->d_emu_counts.ensure((size_t)out_cap * S));
        HIPCHK(c->d_reg_f.ensure((uint64_t)nslots * reg_cap));
        HIPCHK(c->d_reg_r.ensure((uint64_t)nslots * reg_cap));
        HIPCHK(c->d_reg_hit.ensure((uint64_t)nslots * reg_cap));
        HIPCHK(c->d_reg_hits.ensure((uint64_t)nslots * reg_cap * S));
        EmuParams E{};
        E.units = c->d_units.p;
        E.nunits = nu;
        E.unit_buffer = c->d_unit_buffer.p;
        E.gunits = c->d_gunits.p;
        E.goff = c->d_goff.p;
        E.ngroups = ngroups;
        E.unit_head = d_head;
        E.S = S;
        E.nnc = (int32_t)c->nc.size();
        E.nc = c->d_nc.p;
        E.is_control = c->d_ctl.p;
        E.coef = c->d_coef.p;
        E.ncoef = (int32_t)c->coef.size();
        E.kern = c->d_kern.p;
        E.bw = c->p.bw;
        E.nondir = c->p.nondir;
        E.region_thr = c->p.region_thr;
        E.kurt_thr = c->p.kurt_thr;
        E.corr_thr = c->p.corr_thr;
        E.hit_thr = c->p.hit_thr;
        E.want_corr = c->p.want_corr || c->p.corr_thr > -1;
        E.resync = c->d_resync.p;
        E.out = c->d_emu_out.p;
        E.out_counts = c->d_emu_counts.p;
        E.nout = c->d_emu_n.p;
        E.out_cap = out_cap;
        E.ring_hits = c->d_ring_hits.p;
        E.reg_f = c->d_reg_f.p;
        E.reg_r = c->d_reg_r.p;
        E.reg_hit = c->d_reg_hit.p;
        E.reg_hits = c->d_reg_hits.p;
        E.reg_cap = reg_cap;
        E.err = c->d_emu_err.p;
        E.replay_all = replay_all ? 1 : 0;
        E.ring_lds = ring_lds ? 1 : 0;
        E.ring_f = c->d_ring_f.p;
        E.ring_r = c->d_ring_r.p;
        E.ring_has = c->d_ring_has.p;
        E.out_scores = c->d_emu_scores.p;
        E.out_score_off = c->d_emu_score_off.p;
        E.nscores = c->d_emu_nscores.p;
        E.scores_cap = c->d_emu_scores.n;
        if (q) {
            HIPCHK(c->d_emu_group.ensure(out_cap));
            E.q11 = 1;
            E.gskip = c->d_gskip.p;
            E.gstop = c->d_gstop.p;
            E.out_group = c->d_emu_group.p;
            if (ranges) {
                E.gbeg = c->d_gbeg.p;
                E.gend = c->d_gend.p;
            }
        }
        if (c->prof_capture && !q) {
            HIPCHK(c->d_pf_unit.ensure(c->pf_cap));
            HIPCHK(c->d_pf_event.ensure(c->pf_cap));
            HIPCHK(c->d_pf_pos.ensure(c->pf_cap));
            HIPCHK(c->d_pf_score.ensure(c->pf_cap));
            HIPCHK(c->d_pf_n.ensure(1));
            HIPCHK(hipMemsetAsync(c->d_pf_n.p, 0, sizeof(unsigned long long), c->stream));
            E.prof_unit = c->d_pf_unit.p;
            E.prof_event = c->d_pf_event.p;
            E.prof_pos = c->d_pf_pos.p;
            E.prof_score = c->d_pf_score.p;
            E.nprof = c->d_pf_n.p;
            E.prof_cap = c->pf_cap;
        }
        hipLaunchKernelGGL(emulate_kernel, dim3(nslots), dim3(64), ring_lds ? ring_bytes : 0, c->stream, E);
        HIPCHK(hipGetLastError());
        uint32_t nemu = 0, err = 0;
        resync.assign(nu, 0);
        HIPCHK(hipMemcpyAsync(&nemu, c->d_emu_n.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(&err, c->d_emu_err.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(resync.data(), c->d_resync.p, nu * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (err & 4u) {
            fprintf(stderr, "unipeak_hip: exact replay: positions out of order\n");
            return UP_E_ARG;
        }
        if (err & 16u) {  // the -w capture is full
            unsigned long long used = 0;
            HIPCHK(hipMemcpy(&used, c->d_pf_n.p, sizeof used, hipMemcpyDeviceToHost));
            c->pf_cap = std::max<uint64_t>(c->pf_cap * 4, used + used / 4);
            --attempt;  // growth only: the capture has no upper bound of its own
            continue;
        }
        if (err & 11u) {  // 1: a region longer than reg_cap positions, 2: more than out_cap
                          // regions, 8: the region-score slab is full
            if (err & 1u) reg_cap_ref *= 4;
            if (err & 2u) c->emu_out_cap = std::max<uint32_t>(c->emu_out_cap * 4, nemu + nemu / 4);
            if (err & 8u) {
                unsigned long long used = 0;
                HIPCHK(hipMemcpy(&used, c->d_emu_nscores.p, sizeof used, hipMemcpyDeviceToHost));
                c->emu_scores_cap = std::max<uint64_t>(c->emu_scores_cap * 4, used + used / 4);
            }
            continue;
        }
        c->h_resync = resync;
        if (q) {
            q->gstop.resize(2 * (size_t)ngroups);
            q->rgroup.resize(nemu);
            if (ngroups) HIPCHK(hipMemcpy(q->gstop.data(), c->d_gstop.p, 2 * ngroups * 4, hipMemcpyDeviceToHost));
            if (nemu) HIPCHK(hipMemcpy(q->rgroup.data(), c->d_emu_group.p, nemu * 4, hipMemcpyDeviceToHost));
        }
        if (c->prof_capture && !q) {  // the captured retirements, grouped by unit (emission order kept)
            unsigned long long np = 0;
            HIPCHK(hipMemcpy(&np, c->d_pf_n.p, sizeof np, hipMemcpyDeviceToHost));
            std::vector<uint32_t> pu(np), pe(np), pp(np);
            std::vector<double> ps_(np);
            if (np) {
                HIPCHK(hipMemcpy(pu.data(), c->d_pf_unit.p, np * 4, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(pe.data(), c->d_pf_event.p, np * 4, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(pp.data(), c->d_pf_pos.p, np * 4, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(ps_.data(), c->d_pf_score.p, np * 8, hipMemcpyDeviceToHost));
            }
            c->h_pf_off.assign(nu + 1, 0);
            for (uint64_t i = 0; i < np; ++i) ++c->h_pf_off[pu[i] + 1];
            for (uint32_t u = 0; u < nu; ++u) c->h_pf_off[u + 1] += c->h_pf_off[u];
            std::vector<uint64_t> fill(c->h_pf_off.begin(), c->h_pf_off.end() - 1);
            c->h_pf_event.resize(np);
            c->h_pf_pos.resize(np);
            c->h_pf_score.resize(np);
            for (uint64_t i = 0; i < np; ++i) {  // one buffer's entries are in slot order
                const uint64_t k = fill[pu[i]]++;
                c->h_pf_event[k] = pe[i];
                c->h_pf_pos[k] = pp[i];
                c->h_pf_score[k] = ps_[i];
            }
        }
        emu.resize(nemu);
        ecnt.resize((size_t)nemu * S);
        soff.resize(nemu);
        if (nemu) {
            HIPCHK(hipMemcpy(emu.data(), c->d_emu_out.p, nemu * sizeof(up_region), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ecnt.data(), c->d_emu_counts.p, ecnt.size() * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(soff.data(), c->d_emu_score_off.p, nemu * 8, hipMemcpyDeviceToHost));
        }
        return UP_OK;
    }
}

// regions -> the host list (unit-major, emission order within a unit) and,
// if set, the caller's record target
static int publish_host_regions(up_ctx *c, const up_ctx::Pass &ps) {
    c->host_regions = true;
    c->nreg = c->h_regions.size();
    if (ps.target) {  // keep the caller's buffer authoritative
        if (c->nreg > ps.target_cap) return UP_E_NOMEM;
        const uint64_t hdr = c->nreg;
        const size_t cb = c->h_counts.size() * sizeof(uint32_t);
        if (ps.target_hostp) {
            uint8_t *h = (uint8_t *)ps.target_hostp;
            std::memcpy(h, &hdr, 8);
            if (c->nreg) {
                std::memcpy(h + 8, c->h_regions.data(), c->nreg * sizeof(up_region));
                std::memcpy(h + 8 + ps.target_cap * sizeof(up_region), c->h_counts.data(), cb);
            }
        } else {
            HIPCHK(hipMemcpy(ps.target, &hdr, 8, hipMemcpyHostToDevice));
            if (c->nreg) {
                HIPCHK(hipMemcpy(ps.target + 8, c->h_regions.data(), c->nreg * sizeof(up_region), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(ps.target + 8 + ps.target_cap * sizeof(up_region), c->h_counts.data(), cb,
                                 hipMemcpyHostToDevice));
            }
        }
    }
    return UP_OK;
}

// after the pass of `slot` completed (stream idle)
static int replay_head_hits(up_ctx *c, int slot) {
    c->host_regions = false;
    const uint32_t nu = (uint32_t)c->units.size();
    const uint32_t *head = c->hp_head[slot].p;
    bool any = false;
    for (uint32_t i = 0; i < nu; ++i) any |= head[i] != 0;
    c->h_resync.assign(nu, 0);  // no unit replayed (yet)
    c->h_pf_off.assign(nu + 1, 0);
    if (!any) return UP_OK;
    // the head flags are a function of the (unchanged) tracks, so d_head of
    // a later pass still describes this one
    HIPCHK(hipStreamSynchronize(c->stream));
    const int S = c->p.n_samples;
    std::vector<up_region> emu;
    std::vector<uint32_t> ecnt, resync;
    std::vector<uint64_t> soff;
    int rc = emulate_units(c, c->pass[slot].d_head.p, false, emu, ecnt, resync, soff);
    if (rc) return rc;
    const uint32_t nemu = (uint32_t)emu.size();
    // the parallel path's records of this pass, wherever K3 wrote them
    const up_ctx::Pass &ps = c->pass[slot];
    const up_region *par = c->hp_regions[slot].p;
    const uint32_t *pcnt = c->hp_counts[slot].p;
    std::vector<up_region> dpar;
    std::vector<uint32_t> dcnt;
    if (ps.target && ps.target_hostp) {
        par = (const up_region *)((const uint8_t *)ps.target_hostp + 8);
        pcnt = (const uint32_t *)((const uint8_t *)ps.target_hostp + 8 + ps.target_cap * sizeof(up_region));
    } else if (ps.target) {
        dpar.resize(c->nreg);
        dcnt.resize((size_t)c->nreg * S);
        if (c->nreg) {
            HIPCHK(hipMemcpy(dpar.data(), ps.target + 8, c->nreg * sizeof(up_region), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(dcnt.data(), ps.target + 8 + ps.target_cap * sizeof(up_region),
                             dcnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        }
        par = dpar.data();
        pcnt = dcnt.data();
    }
    // merge, unit-major: within a unit the replayed regions (emission
    // order), then the parallel ones that start at or after the resync
    // position.  The parallel records are unit-major already (K2's order):
    // one linear pass, the untouched runs of records copied in bulk
    std::vector<uint32_t> eorder(nemu);
    for (uint32_t i = 0; i < nemu; ++i) eorder[i] = i;
    std::stable_sort(eorder.begin(), eorder.end(), [&](uint32_t a, uint32_t b) { return emu[a].unit < emu[b].unit; });
    c->h_regions.clear();
    c->h_counts.clear();
    c->h_emulated.clear();
    c->h_score_off.clear();
    c->h_regions.reserve(c->nreg + nemu);
    c->h_counts.reserve((c->nreg + nemu) * (size_t)S);
    c->h_emulated.reserve(c->nreg + nemu);
    c->h_score_off.reserve(c->nreg + nemu);
    auto push_par = [&](uint64_t a, uint64_t b) {  // par records [a, b)
        if (a >= b) return;
        c->h_regions.insert(c->h_regions.end(), par + a, par + b);
        c->h_counts.insert(c->h_counts.end(), pcnt + a * S, pcnt + b * S);
        c->h_emulated.insert(c->h_emulated.end(), b - a, 0);
        c->h_score_off.insert(c->h_score_off.end(), b - a, ~0ull);
    };
    uint32_t ei = 0;
    uint64_t pi = 0;
    while (ei < nemu || pi < c->nreg) {
        // the next unit holding a record of either list
        const uint32_t ue = ei < nemu ? emu[eorder[ei]].unit : ~0u;
        const uint32_t up = pi < c->nreg ? par[pi].unit : ~0u;
        const uint32_t u = ue < up ? ue : up;
        for (; ei < nemu && emu[eorder[ei]].unit == u; ++ei) {
            const uint32_t i = eorder[ei];
            c->h_regions.push_back(emu[i]);
            c->h_counts.insert(c->h_counts.end(), ecnt.begin() + (size_t)i * S, ecnt.begin() + (size_t)(i + 1) * S);
            c->h_emulated.push_back(1);
            c->h_score_off.push_back(soff[i]);
        }
        const uint32_t x = u < resync.size() ? resync[u] : 0u;
        uint64_t run = pi;  // start of the current run of kept records
        for (; pi < c->nreg && par[pi].unit == u; ++pi) {
            if (x != 0 && par[pi].left < x) {
                push_par(run, pi);
                run = pi + 1;
            }
        }
        push_par(run, pi);
    }
    return publish_host_regions(c, ps);
}

template <typename T>
static void key_add(std::vector<uint8_t> &k, const T &v) {
    const uint8_t *b = (const uint8_t *)&v;
    k.insert(k.end(), b, b + sizeof(T));
}

// K1x -> K1b -> K2a -> K2b -> K3 of a pass on ps.stream (the timing events
// between them only at timing level 2, never while capturing)
// a K1q pass's records in the reference's form (q11place.hip) on `st`: the
// per-unit placement (with the head chains' edits, or none) and, if
// `scatter`, the copy from K3's stage into the pass's record destination
static int q11_place(up_ctx *c, int slot, hipStream_t st, const Q11Edit *d_edit, bool scatter) {
    up_ctx::Pass &ps = c->pass[slot];
    const uint32_t nu = (uint32_t)c->units.size();
    HIPCHK(c->d_q11_tab.ensure(std::max(nu, 1u)));
    HIPCHK(c->d_q11_scr.ensure(2 * (size_t)std::max(nu, 1u)));
    up_region *out;
    uint32_t *oc;
    uint64_t dcap;
    if (ps.target) {
        out = (up_region *)(ps.target + 8);
        oc = (uint32_t *)(ps.target + 8 + ps.target_cap * sizeof(up_region));
        dcap = ps.target_cap;
    } else {
        out = c->hp_regions[slot].dev;
        oc = c->hp_counts[slot].dev;
        dcap = std::min<uint64_t>(c->hp_regions[slot].n, c->hp_counts[slot].n / (uint64_t)c->p.n_samples);
    }
    hipLaunchKernelGGL(q11_table_kernel, dim3(1), dim3(1024), 0, st, c->d_unit_buffer.p, nu, ps.d_runit.p,
                       ps.d_starts.p, ps.d_nreg.p, d_edit, c->d_q11_tab.p, c->d_q11_scr.p, c->hp_status[slot].dev,
                       (unsigned long long *)ps.target, dcap);
    HIPCHK(hipGetLastError());
    if (!scatter) return UP_OK;
    HIPCHK(c->d_q11_st.ensure(dcap + 1));
    HIPCHK(c->d_q11_en.ensure(dcap + 1));
    HIPCHK(c->d_q11_src.ensure(dcap + 1));
    const unsigned blocks = (unsigned)std::min<uint64_t>((ps.cap + 255) / 256 + 1, 4096);
    hipLaunchKernelGGL(q11_scatter_kernel, dim3(blocks), dim3(256), 0, st, c->d_q11_stage.p,
                       c->d_q11_stage_cnt.p, ps.d_nreg.p, (int)c->p.n_samples, c->d_q11_tab.p, out, oc, dcap,
                       c->d_q11_st.p, c->d_q11_en.p, c->d_q11_src.p);
    HIPCHK(hipGetLastError());
    return UP_OK;
}

static int enqueue_rest(up_ctx *c, int slot, const ScanParams &SP, const StatParams &P, uint64_t cap,
                        uint32_t k1a_waves, uint32_t k1a_xcap, bool events) {
    up_ctx::Pass &ps = c->pass[slot];
    const uint32_t ns = c->nstrips;
    const uint32_t nsb = (ns + kSegBlock - 1) / kSegBlock;
    if (!ps.req_q11 && c->p.bw <= kMaxBw) {  // (K1q and K1w wrote every strip's runs themselves)
        if (k1a_waves) {  // K1x: list the stashed work-list entries for K1b
            hipLaunchKernelGGL(xref_kernel, dim3(1), dim3(1024), 0, ps.stream, ps.d_xwcount.p, k1a_waves,
                               k1a_xcap, ps.d_xref.p, ps.d_xcount.p);
            HIPCHK(hipGetLastError());
        }
        dispatch_scan<false, kModeExact>(c, ps.stream, SP, 0, ns);    // K1b: exact blocks
        HIPCHK(hipGetLastError());
    }
    if (events) HIPCHK(hipEventRecord(ps.ev[2], ps.stream));
    unsigned long long *thdr = (unsigned long long *)ps.target;
    if (int r = launch_seg_count_head(c, slot)) return r;
    hipLaunchKernelGGL(seg_compact_kernel, dim3(nsb), dim3(kSegBlock), 0, ps.stream, c->d_units.p,
                       (uint32_t)c->units.size(), ps.d_info.p, ps.d_cnt.p, ps.d_bsum.p, ps.d_rec.p,
                       ps.d_ovf_rec.p, ps.ovf_cap, ps.d_starts.p, ps.d_ends.p, ps.d_runit.p, ps.d_peak_pos.p,
                       ps.d_peak_val.p, ns, (uint64_t)cap, ps.d_ovf_count.p, ps.d_xcount.p, ps.d_nreg.p,
                       c->hp_status[slot].dev, thdr);
    HIPCHK(hipGetLastError());
    if (events) HIPCHK(hipEventRecord(ps.ev[3], ps.stream));
    dispatch_stats(c, ps.stream, P, std::max<uint64_t>(ps.req_last_nreg, 1024));
    HIPCHK(hipGetLastError());
    if (ps.req_q11_place)
        if (int r = q11_place(c, slot, ps.stream, nullptr, true)) return r;
    if (events) HIPCHK(hipEventRecord(ps.ev[4], ps.stream));
    return UP_OK;
}

// Enqueue one pass K1a -> K1x -> K1b -> K2a -> K2b -> K3 into `slot` with no
// host round trip: the region count stays on the device, the record areas
// are pre-sized (reg_cap, ovf_cap) and K3 writes the records straight into
// mapped pinned host memory (or the caller's record target).  An undersized
// area is detected when the pass is finished; it is grown and the pass rerun
// (first passes only).  K1a is launched directly (between its timing
// events); K1x..K3 go out as one cached hipGraph of the slot.
static int launch_pass(up_ctx *c, int slot) {
    const uint32_t ns = c->nstrips;
    const int S = c->p.n_samples;
    up_ctx::Pass &ps = c->pass[slot];
    const uint32_t nsb = (ns + kSegBlock - 1) / kSegBlock;
    HIPCHK(ps.d_info.ensure(ns));
    HIPCHK(ps.d_rec.ensure((size_t)ns * kRecStride));
    HIPCHK(ps.d_xlist.ensure(((size_t)ns + kMaxK1aWaves) * kXEntry));  // K1a stash regions
    HIPCHK(ps.d_xwcount.ensure(2 * kMaxK1aWaves));
    HIPCHK(ps.d_xref.ensure(ns));
    HIPCHK(ps.d_spk.ensure((size_t)ns * 4));
    HIPCHK(ps.d_cnt.ensure(ns));
    HIPCHK(ps.d_bsum.ensure(nsb));
    HIPCHK(ps.d_nreg.ensure(1));
    HIPCHK(c->hp_status[slot].ensure(4));
    if (!ps.d_xcount.p || !ps.d_ovf_count.p) ps.counters_armed = false;
    HIPCHK(ps.d_xcount.ensure(2));  // front / back ends of the work list
    HIPCHK(ps.d_ovf_count.ensure(1));
    // every per-pass decision reads the request snapshot (ps.req_*), never
    // the live context: the caller may change the record target or grow the
    // capacities while this pass waits for the launcher thread
    const uint64_t cap = ps.req_reg_cap;
    const uint32_t ovf_cap = ps.req_ovf_cap;
    HIPCHK(ps.d_ovf_rec.ensure((size_t)ovf_cap * kOvfStride));
    HIPCHK(ps.d_peak_pos.ensure(cap + 1));
    HIPCHK(ps.d_peak_val.ensure(cap + 1));
    HIPCHK(ps.d_starts.ensure(cap + 1));
    HIPCHK(ps.d_ends.ensure(cap + 1));
    HIPCHK(ps.d_runit.ensure(cap + 1));
    HIPCHK(ps.d_head.ensure(c->units.size()));
    HIPCHK(c->hp_head[slot].ensure(c->units.size()));
    // K3's per-wave (f, r) slabs when the strand correlation is evaluated:
    // at most 8 resident 4-wave workgroups per CU
    const bool corr = c->p.nondir && (c->p.want_corr || c->p.corr_thr > -1);
    const uint32_t corr_cap = 1024;
    if (corr) HIPCHK(ps.d_corr.ensure((size_t)(c->ncu > 0 ? c->ncu : 256) * 8 * 4 * corr_cap * 2));
    if (!ps.req_target) {
        HIPCHK(c->hp_regions[slot].ensure(cap + 1));
        HIPCHK(c->hp_counts[slot].ensure((cap + 1) * S));
    }
    ps.target = ps.req_target;
    ps.target_hostp = ps.req_target_hostp;
    ps.target_cap = ps.req_target_cap;
    ps.cap = cap;
    ps.ovf_cap = ovf_cap;
    // the pass follows everything enqueued on the context stream (track
    // writes), and its K1a follows the K1a of the previous pass if that one
    // is in flight: one streaming K1a at a time, earlier passes' K1b/K2/K3
    // beside it
    // (stream order serialises the K1a's; a slot is reused only after the
    // host saw its previous pass done)
    hipStream_t s1 = c->k1a_stream;
    ps.stream = c->chain[c->nlaunch++ % (uint64_t)c->n_chain];
    // (nothing to follow once the context stream has drained: two API
    // calls per pass fewer, ~5 us of host time, which bounds 8-GPU steps)
    if (hipStreamQuery(c->stream) != hipSuccess) {
        HIPCHK(hipEventRecord(c->host_work, c->stream));
        HIPCHK(hipStreamWaitEvent(s1, c->host_work, 0));
    }
    if (!ps.counters_armed) {  // K2b re-arms them at the end of every pass
        HIPCHK(hipMemsetAsync(ps.d_ovf_count.p, 0, sizeof(uint32_t), s1));
        HIPCHK(hipMemsetAsync(ps.d_xcount.p, 0, 2 * sizeof(uint32_t), s1));
    }
    ScanParams SP = scan_params(c, ps, ovf_cap);
    // K1x..K3 as a captured graph only when the caller's thread launches:
    // capturing on the launcher thread while the caller waits on earlier
    // passes invalidated captures (hipErrorStreamCaptureInvalidated, ROCm
    // 7.2, even in relaxed mode), and off the caller's thread the five
    // plain launches cost nothing on the caller's critical path
    bool graph = c->use_graphs && !c->use_launcher;
#if defined(UPK_DEBUG_COUNTS) || defined(UPK_DEBUG_TIMES)
    static const bool dbg = getenv("UNIPEAK_DEBUG_COUNTS") != nullptr;
    if (dbg) {
        HIPCHK(c->d_dbg.ensure(32));
        HIPCHK(hipMemsetAsync(c->d_dbg.p, 0, 32 * sizeof(unsigned long long), s1));
        SP.dbg = c->d_dbg.p;
        graph = false;
    }
#endif
    ps.tl = ps.req_tl;
    StatParams P = stat_params(c, ps);
    P.cap = cap;
    P.peak_pos = ps.d_peak_pos.p;
    P.peak_val = ps.d_peak_val.p;
    P.spk = ps.d_spk.p;
    P.corr_scratch = corr ? ps.d_corr.p : nullptr;
    P.corr_cap = corr_cap;
    // K3 writes the records straight into mapped pinned host memory (or the
    // caller's record target).  Staging them in device memory and delivering
    // them with DMA copies measured slower twice (round 1: within noise with
    // a second stream; round 3, same box, two rounds each: 4,237 vs 4,405
    // Gbp/s, K3 + copies 0.203 vs 0.167 ms), so there is one delivery path.
    if (ps.target) {  // records into the caller's buffer instead
        P.cap = std::min<uint64_t>(cap, ps.target_cap);
        P.out = (up_region *)(ps.target + 8);
        P.out_counts = (uint32_t *)(ps.target + 8 + ps.target_cap * sizeof(up_region));
    } else {
        P.out = c->hp_regions[slot].dev;
        P.out_counts = c->hp_counts[slot].dev;
    }
    ps.counters_armed = true;  // K2b re-arms them
    const int tl = ps.tl;
    if (tl >= 1) HIPCHK(hipEventRecord(ps.ev[0], s1));
    c->k1a_waves = 0;
    if (ps.req_q11) {  // K1q: runs of processed positions (threshold <= 0)
        graph = false;
        P.peak_pos = nullptr;  // K3 runs its KDE for the peaks
        P.peak_val = nullptr;
        P.q11 = 1;
        // K3 -> the device stage; q11place.hip places the records
        HIPCHK(c->d_q11_stage.ensure(cap + 1));
        HIPCHK(c->d_q11_stage_cnt.ensure((cap + 1) * S));
        P.out = c->d_q11_stage.p;
        P.out_counts = c->d_q11_stage_cnt.p;
        P.cap = cap;
        const unsigned blocks = (unsigned)std::min<uint64_t>((ns + 3) / 4, 4096);
        hipLaunchKernelGGL(proc_runs_kernel, dim3(std::max(1u, blocks)), dim3(256), 0, s1, SP);
    } else {
        if (c->p.bw > kMaxBw) {  // K1w: screen + exact in one (wide.hip)
            graph = false;
            const unsigned blocks = std::max(1u, std::min<uint32_t>(ns, 8192));
            const int pm = pool_mode(c);
            if (pm == 0) hipLaunchKernelGGL(wide_kernel<0>, dim3(blocks), dim3(64), 0, s1, SP);
            else if (pm == 1) hipLaunchKernelGGL(wide_kernel<1>, dim3(blocks), dim3(64), 0, s1, SP);
            else hipLaunchKernelGGL(wide_kernel<2>, dim3(blocks), dim3(64), 0, s1, SP);
        } else {
            // K1a: stream + screen -- the chunk-sum plane when the index is
            // on, else the 2-bit fields (one-pass cost: no derived data read)
            if (plane_scan(c) || window_nh(c->p.bw) > 4) dispatch_scan<false, kModeScreen>(c, s1, SP, 0, ns);
            else dispatch_scan<false, kModeScreenF>(c, s1, SP, 0, ns);
        }
    }
    HIPCHK(hipGetLastError());
    hipEvent_t k1a_end = ps.k1a_end;  // a timed pass's end-of-K1a event serves as well
    if (tl >= 1) k1a_end = ps.ev[1];
    HIPCHK(hipEventRecord(k1a_end, s1));
    HIPCHK(hipStreamWaitEvent(ps.stream, k1a_end, 0));
    const uint32_t kw = c->k1a_waves, kx = c->k1a_xcap;
    if (!graph || tl >= 2) {
        if (int r = enqueue_rest(c, slot, SP, P, cap, kw, kx, tl >= 2)) return r;
        HIPCHK(hipEventRecord(ps.done, ps.stream));
        return UP_OK;
    }
    // every launch argument of K1x..K3: parameter blocks and grid inputs
    std::vector<uint8_t> key;
    key_add(key, SP);
    key_add(key, P);
    key_add(key, kw);
    key_add(key, kx);
    key_add(key, std::max<uint64_t>(ps.req_last_nreg, 1024));
    key_add(key, (uint32_t)c->units.size());
    key_add(key, ovf_cap);
    key_add(key, pool_mode(c));
    key_add(key, c->p.nondir);
    key_add(key, c->nc.size());
    key_add(key, c->hp_head[slot].dev);
    key_add(key, c->hp_status[slot].dev);
    key_add(key, ps.d_head.p);
    key_add(key, c->d_coef.p);
    key_add(key, ps.target);
    key_add(key, ps.d_cnt.p);
    key_add(key, ps.d_bsum.p);
    size_t gi = 0;
    while (gi < ps.graphs.size() && ps.graphs[gi].first != key) ++gi;
    if (gi == ps.graphs.size()) {
        HIPCHK(hipStreamBeginCapture(ps.stream, hipStreamCaptureModeThreadLocal));
        const int r = enqueue_rest(c, slot, SP, P, cap, kw, kx, false);
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(ps.stream, &g);
        if (r) {
            if (g) (void)hipGraphDestroy(g);
            return r;
        }
        HIPCHK(e);
        hipGraphExec_t x = nullptr;
        const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        HIPCHK(ei);
        if (ps.graphs.size() >= 8) {  // keep the most recent ones
            (void)hipGraphExecDestroy(ps.graphs.back().second);
            ps.graphs.pop_back();
        }
        ps.graphs.insert(ps.graphs.begin(), {key, x});
        gi = 0;
    }
    HIPCHK(hipGraphLaunch(ps.graphs[gi].second, ps.stream));
    HIPCHK(hipEventRecord(ps.done, ps.stream));
    return UP_OK;
}

static int prepare_run(up_ctx *c) {
    int r = check_runnable(c);
    if (r) return r;
    HIPCHK(hipSetDevice(c->dev));
    return sync_units(c);
}

static void launcher_main(up_ctx *c) {
    (void)hipSetDevice(c->dev);
    std::unique_lock<std::mutex> lk(c->lmu);
    for (;;) {
        c->lcv.wait(lk, [&] { return c->lstop || !c->lq.empty(); });
        if (c->lq.empty()) return;  // stopping, nothing queued
        const int slot = c->lq.front();
        c->lq.pop_front();
        c->lbusy = true;
        lk.unlock();
        const int r = launch_pass(c, slot);
        lk.lock();
        c->pass[slot].lrc = r;
        c->pass[slot].lpending = false;
        c->lbusy = false;
        c->lcv.notify_all();
    }
}

// every queued pass launched (the launcher idle)
static void launcher_drain(up_ctx *c) {
    std::unique_lock<std::mutex> lk(c->lmu);
    c->lcv.wait(lk, [&] { return c->lq.empty() && !c->lbusy; });
}

static void settle_in_flight(up_ctx *c) {
    launcher_drain(c);
    sync_all(c);
}

static void launcher_stop(up_ctx *c) {
    if (!c->launcher.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(c->lmu);
        c->lstop = true;
    }
    c->lcv.notify_all();
    c->launcher.join();
}

int up_run_async(up_ctx *c) {
    if (!c) return UP_E_ARG;
    if (c->seq_launched - c->seq_done >= kSlots) return UP_E_STATE;  // at most kSlots passes in flight
    if (busy(c) && c->units_dirty) return UP_E_STATE;  // passes in flight read the unit table
    int r = prepare_run(c);
    if (r) return r;
    const int slot = (int)(c->seq_launched % kSlots);
    up_ctx::Pass &ps = c->pass[slot];
    ps.t0 = std::chrono::steady_clock::now();
    ps.lrc = 0;
    if (c->units.empty()) {
        ++c->seq_launched;
        return UP_OK;
    }
    ps.req_target = c->target;
    ps.req_target_hostp = c->target_hostp;
    ps.req_target_cap = c->target_cap;
    ps.req_tl = c->timing;
    ps.req_q11 = c->q11_run;
    ps.req_q11_place = c->q11_run && c->q11_place_in_pass;
    ps.req_last_nreg = c->last_nreg;
    ps.req_reg_cap = c->reg_cap;
    ps.req_ovf_cap = c->ovf_cap;
    if (c->use_launcher) {
        if (!c->launcher.joinable()) c->launcher = std::thread(launcher_main, c);
        {
            std::lock_guard<std::mutex> lk(c->lmu);
            ps.lpending = true;
            c->lq.push_back(slot);
        }
        c->lcv.notify_one();
    } else if ((r = launch_pass(c, slot))) {
        sync_all(c);
        c->seq_done = c->seq_launched;  // drop whatever was in flight
        return r;
    }
    ++c->seq_launched;
    ++c->passes_on_tracks;
    return UP_OK;
}

// complete the oldest pass in flight
int up_run_wait(up_ctx *c, uint64_t *n_regions) {
    if (!c) return UP_E_ARG;
    if (!busy(c)) return UP_E_STATE;
    HIPCHK(hipSetDevice(c->dev));
    const int slot = (int)(c->seq_done % kSlots);
    up_ctx::Pass &ps = c->pass[slot];
    c->ran = false;
    c->nreg = 0;
    c->host_regions = false;
    c->q11_placed = false;
    c->cur_slot = slot;
    if (c->units.empty()) {
        ++c->seq_done;
        if (n_regions) *n_regions = 0;
        c->ran = true;
        return UP_OK;
    }
    auto fail = [&](int rc) {
        launcher_drain(c);
        sync_all(c);
        c->seq_done = c->seq_launched;
        return rc;
    };
    {   // the launcher thread has enqueued this pass
        std::unique_lock<std::mutex> lk(c->lmu);
        c->lcv.wait(lk, [&] { return !ps.lpending; });
    }
    if (ps.lrc) return fail(ps.lrc);
    if (hipEventSynchronize(ps.done) != hipSuccess) return fail(UP_E_HIP);
    uint64_t nreg = 0;
    for (int attempt = 0;; ++attempt) {
        if (attempt == 3) return fail(UP_E_INTERNAL);
        const unsigned long long *st = c->hp_status[slot].p;
        if (st[2]) return fail(UP_E_INTERNAL);  // starts and ends disagree
        nreg = st[0];
        const uint64_t ovf = st[1];
        bool again = false;
        if (ovf > ps.ovf_cap) { c->ovf_cap = std::max<uint32_t>(c->ovf_cap, (uint32_t)(ovf + ovf / 2 + 64)); again = true; }
        if (nreg > ps.cap) { c->reg_cap = std::max<uint64_t>(c->reg_cap, nreg + nreg / 4 + 1024); again = true; }
        if (ps.target && nreg > ps.target_cap) return fail(UP_E_NOMEM);  // caller's buffer too small
#if defined(UPK_DEBUG_COUNTS) || defined(UPK_DEBUG_TIMES)
        if (getenv("UNIPEAK_DEBUG_COUNTS")) {
            unsigned long long h[32];
            HIPCHK(hipMemcpy(h, c->d_dbg.p, sizeof h, hipMemcpyDeviceToHost));
            fprintf(stderr, "unipeak_hip: K1 strips %u exact blocks %llu live words %llu hits %llu "
                            "cycles load %llu scatter %llu; words with a flag %llu, flagged positions %llu, "
                            "words reaching thr/2 %llu\n",
                    c->nstrips, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
            fprintf(stderr, "unipeak_hip: K1b clocks: item %llu load %llu scatter %llu flags %llu items %llu "
                            "max wave %llu waves %llu (Q part of scatter %llu)\n", h[16], h[17], h[18], h[19],
                    h[20], h[21], h[22], h[23]);
            fprintf(stderr, "unipeak_hip: K1b items by exact blocks:");
            for (int k = 1; k <= 16; ++k) fprintf(stderr, " %d:%llu", k, h[8 + k]);
            fprintf(stderr, "\n");
        }
#endif
        if (!again) break;
        // rerun this pass alone with grown areas (a later pass in flight
        // finishes first; its own status tells whether it needs the same)
        // (the launcher first enqueues what is queued: this thread then owns
        // the launch state)
        launcher_drain(c);
        if (hipDeviceSynchronize() != hipSuccess) return fail(UP_E_HIP);
        ps.req_reg_cap = c->reg_cap;   // the grown areas; same record target and timing
        ps.req_ovf_cap = c->ovf_cap;
        int r = launch_pass(c, slot);
        if (r) return fail(r);
        if (hipEventSynchronize(ps.done) != hipSuccess) return fail(UP_E_HIP);
    }
    c->nreg = nreg;
    c->last_nreg = nreg;
    // (a K1q pass's head units take q11_finish's chains instead)
    int r = ps.req_q11 ? UP_OK : replay_head_hits(c, slot);
    if (r) return fail(r);
    const int tl = ps.tl;
    float a = 0, b = 0, d = 0, x = 0;
    if (tl >= 1) (void)hipEventElapsedTime(&a, ps.ev[0], ps.ev[1]);
    if (tl >= 2) {
        (void)hipEventElapsedTime(&x, ps.ev[1], ps.ev[2]);
        (void)hipEventElapsedTime(&b, ps.ev[2], ps.ev[3]);
        (void)hipEventElapsedTime(&d, ps.ev[3], ps.ev[4]);
    }
    c->times[0] = (double)a + x;  // K1 = K1a + K1b (K1a alone when only it is timed)
    c->times[4] = x;              // K1b share of K1
    c->times[1] = b;
    c->times[2] = d;
    c->times[3] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ps.t0).count();
    ++c->seq_done;
    c->ran = true;
    if (n_regions) *n_regions = c->nreg;
    return UP_OK;
}

// The segmented replay (round 5): configurations outside the parallel scan
// still replay every position exactly, but as independent chains, one from
// each run start (leap_adds_kernel: an add with no add in the 2bw + 1
// positions before it, where the window has drained and a fresh state is
// the true one), each stopping at the first leap past its start that closes
// the open region over a clean window (the q11 chains' rule).  A chain that
// reaches past the next chain's start (an unclean window: quirk Q1 leftovers,
// a region carried across a unit boundary) covers it, and that chain is
// dropped.  Records: the kept chains', unit-major, in emission order.
static int replay_segments(up_ctx *c, std::vector<up_region> &emu, std::vector<uint32_t> &ecnt,
                           std::vector<uint64_t> &soff, std::vector<uint32_t> &keep) {
    const uint32_t nu = (uint32_t)c->units.size();
    const int S = c->p.n_samples;
    const int bw = c->p.bw;
    std::vector<unsigned long long> starts;
    for (int attempt = 0;; ++attempt) {
        HIPCHK(c->d_seg.ensure(c->seg_cap));
        HIPCHK(c->d_seg_n.ensure(1));
        HIPCHK(hipMemsetAsync(c->d_seg_n.p, 0, 4, c->stream));
        const unsigned blocks = std::max(1u, std::min<uint32_t>((c->nstrips + 3) / 4, 4096));
        hipLaunchKernelGGL(leap_adds_kernel, dim3(blocks), dim3(256), 0, c->stream, c->d_units.p, nu, c->nstrips,
                           S, bw, c->d_seg.p, c->d_seg_n.p, c->seg_cap);
        HIPCHK(hipGetLastError());
        uint32_t n = 0;
        HIPCHK(hipMemcpyAsync(&n, c->d_seg_n.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (n > c->seg_cap) {
            if (attempt) return UP_E_INTERNAL;
            c->seg_cap = n + n / 4 + 1024;
            continue;
        }
        starts.resize(n);
        if (n) HIPCHK(hipMemcpy(starts.data(), c->d_seg.p, (size_t)n * 8, hipMemcpyDeviceToHost));
        break;
    }
    std::sort(starts.begin(), starts.end());  // (unit, position)
    std::vector<uint32_t> order[2], at(nu);
    for (uint32_t u = 0; u < nu; ++u) {
        at[u] = (uint32_t)order[c->units[u].buffer].size();
        order[c->units[u].buffer].push_back(u);
    }
    Q11Chains q;
    uint32_t base[2];
    for (int b = 0; b < 2; ++b) {
        base[b] = (uint32_t)q.gunits.size();
        q.gunits.insert(q.gunits.end(), order[b].begin(), order[b].end());
    }
    struct G { int b; uint32_t k0; int64_t s; };
    std::vector<G> gs;
    gs.reserve(starts.size());
    for (unsigned long long e : starts) {
        const uint32_t u = (uint32_t)(e >> 32), a = (uint32_t)e;
        const int b = c->units[u].buffer;
        q.gbeg.push_back(base[b] + at[u]);
        q.gend.push_back(base[b] + (uint32_t)order[b].size());
        q.gskip.push_back(a);
        gs.push_back(G{b, at[u], (int64_t)a - bw});
    }
    std::vector<uint32_t> resync;
    up_ctx::Pass &p0 = c->pass[0];
    if (int r = emulate_units(c, p0.d_head.p, true, emu, ecnt, resync, soff, &q)) return r;
    std::vector<uint8_t> kept(gs.size(), 0);
    int64_t last[2] = {-1, -1};
    for (size_t g = 0; g < gs.size(); ++g) {
        const G &G_ = gs[g];
        if (last[G_.b] >= 0) {
            const size_t l = (size_t)last[G_.b];
            if (q.gstop[2 * l] == ~0u) continue;  // ran to the buffer's end
            const uint32_t sk = at[q.gstop[2 * l]];
            if (sk > G_.k0 || (sk == G_.k0 && (int64_t)q.gstop[2 * l + 1] > G_.s)) continue;  // covered
        }
        kept[g] = 1;
        last[G_.b] = (int64_t)g;
    }
    keep.clear();
    for (uint32_t i = 0; i < emu.size(); ++i)
        if (kept[q.rgroup[i]]) keep.push_back(i);
    std::stable_sort(keep.begin(), keep.end(), [&](uint32_t x, uint32_t y) {
        if (emu[x].unit != emu[y].unit) return emu[x].unit < emu[y].unit;
        return q.rgroup[x] < q.rgroup[y];
    });
    return UP_OK;
}

// every unit through K0 (replay_mode configurations): the segmented replay,
// or -- with the -w capture on (its retirements must keep each unit's add
// order) or UNIPEAK_REPLAY_WHOLE=1 -- one chain per buffer, never resynced
static int run_replay(up_ctx *c, uint64_t *n_regions) {
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(c->dev));
    c->ran = false;
    c->nreg = 0;
    c->host_regions = false;
    c->q11_placed = false;
    c->h_regions.clear();
    c->h_counts.clear();
    c->h_emulated.clear();
    c->h_score_off.clear();
    int r = sync_units(c);
    if (r) return r;
    const uint32_t nu = (uint32_t)c->units.size();
    c->h_resync.assign(nu, 0);
    c->h_pf_off.assign(nu + 1, 0);
    up_ctx::Pass ps;
    ps.target = c->target;
    ps.target_hostp = c->target_hostp;
    ps.target_cap = c->target_cap;
    if (nu) {
        up_ctx::Pass &p0 = c->pass[0];  // no pass in flight (replay configurations)
        HIPCHK(p0.d_head.ensure(nu));
        HIPCHK(hipMemsetD32Async((hipDeviceptr_t)p0.d_head.p, 1, nu, c->stream));
        std::vector<up_region> emu;
        std::vector<uint32_t> ecnt, resync;
        std::vector<uint64_t> soff;
        std::vector<uint32_t> order;
        static const bool whole = [] {
            const char *e = getenv("UNIPEAK_REPLAY_WHOLE");
            return e && *e == '1';
        }();
        // (the segmented replay's chains assume a window drained after 2bw + 1
        // positions without an add: false from bw 32,768 on, where the
        // reference's UShort retirement count wraps -- wide_mode)
        if (!c->prof_capture && kTB == 2 && !whole && c->p.bw <= kMaxWideBw) {
            if ((r = replay_segments(c, emu, ecnt, soff, order))) return r;
            c->h_resync.assign(nu, 0);
        } else {
            if ((r = emulate_units(c, p0.d_head.p, true, emu, ecnt, resync, soff))) return r;
            order.resize(emu.size());
            for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
            std::stable_sort(order.begin(), order.end(),
                             [&](uint32_t a, uint32_t b) { return emu[a].unit < emu[b].unit; });
        }
        const int S = c->p.n_samples;
        for (uint32_t i : order) {
            c->h_regions.push_back(emu[i]);
            c->h_counts.insert(c->h_counts.end(), ecnt.begin() + (size_t)i * S, ecnt.begin() + (size_t)(i + 1) * S);
            c->h_emulated.push_back(1);
            c->h_score_off.push_back(soff[i]);
        }
    }
    if ((r = publish_host_regions(c, ps))) return r;
    for (double &t : c->times) t = 0;
    c->times[3] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->ran = true;
    if (n_regions) *n_regions = c->nreg;
    return UP_OK;
}

// the records of a K1q pass -> the reference's regions, placed on the device
// (q11place.hip; without heads already inside the pass):
//  * every run [s, e] was reached by a leap: Region::left = s + 1, right =
//    e + 1, peak = (first maximum over s + 1 .. e) + 1 (K3 skipped s), its
//    statistics over s .. e as K3 computed them (peakcall.cpp:76-78,
//    data.cpp:92-102); closed by the add after the first add at pos >=
//    right + bw + 1, else by the flush (UP_CLOSE_Q11);
//  * the last run of a unit is still open after its flush: the buffer's
//    next unit relabels it (peakcall.cpp:164-168) and its first leap closes
//    it -- the record moves there (UP_CLOSE_Q11_HEAD, positions still the
//    previous unit's); the buffer's last unit's last run is never closed;
//  * heads (units with an add at <= bw + 1, which process position 1 --
//    continuing the open region across the unit boundary -- or land the
//    misaligned window of quirk Q1): the exact replay (K0) covers each one
//    from the start of the buffer's previous unit's last run (a leap: the
//    window there holds only that add, so a fresh state is exact) to the
//    first leap past the head that closes the open region over a clean
//    window (Q11Chains); K1q's records before that leap and the moved one
//    give way to the replay's, those from the leap on stay (Q11Edit).  A
//    chain that reaches a later head's start point covers it too (that
//    head's own chain is dropped).
static int q11_finish(up_ctx *c, const std::vector<uint32_t> *heads) {
    const int slot = c->cur_slot;
    up_ctx::Pass &ps = c->pass[slot];
    const int S = c->p.n_samples;
    const uint32_t nu = (uint32_t)c->units.size();
    c->host_regions = false;
    c->q11_placed = true;
    c->q11_rep.clear();
    c->h_resync.assign(nu, 0);
    c->h_pf_off.assign(nu + 1, 0);
    const unsigned long long *st = c->hp_status[slot].p;
    if (!heads) {  // placed inside the pass
        // (no unit: no pass ran, and st[3] may still hold an earlier pass's count)
        c->nreg = (nu && st[3]) ? st[3] - 1 : 0;
        return UP_OK;
    }
    // each unit's K1q records (the placement table without edits)
    HIPCHK(hipStreamSynchronize(ps.stream));
    if (int r = q11_place(c, slot, c->stream, nullptr, false)) return r;
    std::vector<Q11Place> tab(nu);
    HIPCHK(hipMemcpyAsync(tab.data(), c->d_q11_tab.p, nu * sizeof(Q11Place), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    // the chains: one per head, from the start of the buffer's previous unit
    // with records' last run (its raw start s: the add at s + bw begins it)
    struct G { int b; uint32_t k0; uint64_t s; };  // buffer, start index in its order, run start (0: fresh)
    std::vector<G> gs;
    Q11Chains q;
    std::vector<uint32_t> order[2];
    for (uint32_t u = 0; u < nu; ++u) order[c->units[u].buffer].push_back(u);
    for (int b = 0; b < 2; ++b) {
        const std::vector<uint32_t> &o = order[b];
        int64_t pw = -1;  // the previous unit with records (index into o)
        for (uint32_t k = 0; k < o.size(); ++k) {
            const uint32_t u = o[k];
            if ((*heads)[u]) {
                G g{b, k, 0};
                uint32_t skip = 1;
                if (pw >= 0) {
                    const uint32_t pu = o[(size_t)pw];
                    uint32_t s0 = 0;
                    HIPCHK(hipMemcpy(&s0, ps.d_starts.p + tab[pu].first + tab[pu].cnt - 1, 4, hipMemcpyDeviceToHost));
                    g.k0 = (uint32_t)pw;
                    g.s = s0;
                    skip = (uint32_t)(g.s + c->p.bw);
                }
                q.gunits.insert(q.gunits.end(), o.begin() + g.k0, o.end());
                q.goff.push_back((uint32_t)q.gunits.size());
                q.gskip.push_back(skip);
                gs.push_back(g);
            }
            if (tab[u].cnt) pw = k;
        }
    }
    std::vector<up_region> emu;
    std::vector<uint32_t> ecnt, resync;
    std::vector<uint64_t> soff;
    if (int r = emulate_units(c, c->d_q11_head.p, true, emu, ecnt, resync, soff, &q)) return r;
    c->h_resync.assign(nu, 0);
    // keep a chain unless an earlier kept chain of its buffer reached past
    // its start point; the edits of the kept ones
    std::vector<Q11Edit> ed(nu, Q11Edit{0u, 0xFFFFFFFFu, 0u, 0u});
    std::vector<uint8_t> kept(gs.size(), 0);
    int64_t last[2] = {-1, -1};
    for (size_t g = 0; g < gs.size(); ++g) {
        const G &G_ = gs[g];
        const std::vector<uint32_t> &o = order[G_.b];
        if (last[G_.b] >= 0) {
            const size_t l = (size_t)last[G_.b];
            if (q.gstop[2 * l] == ~0u) continue;  // ran to the buffer's end
            const uint32_t sk = (uint32_t)(std::find(o.begin(), o.end(), q.gstop[2 * l]) - o.begin());
            if (sk > G_.k0 || (sk == G_.k0 && q.gstop[2 * l + 1] > G_.s)) continue;  // covered
        }
        kept[g] = 1;
        last[G_.b] = (int64_t)g;
        const bool stopped = q.gstop[2 * g] != ~0u;
        const uint32_t sk = stopped ? (uint32_t)(std::find(o.begin(), o.end(), q.gstop[2 * g]) - o.begin())
                                    : (uint32_t)o.size();
        uint32_t k = G_.k0;
        if (G_.s) ed[o[k++]].hi = (uint32_t)G_.s;
        for (; k < sk; ++k) ed[o[k]].flags |= kQ11Full;
        if (stopped) {
            ed[q.gstop[2 * g]].lo = q.gstop[2 * g + 1];
            ed[q.gstop[2 * g]].flags |= kQ11NoMove;
        }
    }
    // the kept chains' records per unit, in emission order
    std::vector<std::vector<uint32_t>> rep(nu);
    for (uint32_t i = 0; i < emu.size(); ++i)
        if (kept[q.rgroup[i]]) rep[emu[i].unit].push_back(i);
    for (uint32_t u = 0; u < nu; ++u) ed[u].nrep = (uint32_t)rep[u].size();
    HIPCHK(c->d_q11_edit.ensure(std::max(nu, 1u)));
    HIPCHK(hipMemcpy(c->d_q11_edit.p, ed.data(), nu * sizeof(Q11Edit), hipMemcpyHostToDevice));
    // place K1q's records around the replayed ones (growing the pinned
    // record area when the replay adds more than K1q dropped)
    uint64_t total = 0;
    for (int attempt = 0;; ++attempt) {
        if (int r = q11_place(c, slot, c->stream, c->d_q11_edit.p, true)) return r;
        HIPCHK(hipStreamSynchronize(c->stream));
        total = st[3] ? st[3] - 1 : 0;
        const uint64_t dcap = ps.target ? ps.target_cap
                                        : std::min<uint64_t>(c->hp_regions[slot].n, c->hp_counts[slot].n / (uint64_t)S);
        if (total <= dcap) break;
        if (ps.target || attempt) return UP_E_NOMEM;
        HIPCHK(c->hp_regions[slot].ensure(total + 1));
        HIPCHK(c->hp_counts[slot].ensure((total + 1) * S));
        st = c->hp_status[slot].p;
    }
    // the replayed records into their slots: after the unit's moved-in one
    std::vector<uint64_t> scr(2 * (size_t)nu);
    HIPCHK(hipMemcpy(scr.data(), c->d_q11_scr.p, scr.size() * 8, hipMemcpyDeviceToHost));
    for (uint32_t u = 0; u < nu; ++u) {
        uint64_t d = scr[2 * u] + (scr[2 * u + 1] & 1u);
        for (uint32_t i : rep[u]) {
            const up_region &r = emu[i];
            const uint32_t *k = ecnt.data() + (size_t)i * S;
            if (ps.target && ps.target_hostp) {
                uint8_t *h = (uint8_t *)ps.target_hostp;
                std::memcpy(h + 8 + d * sizeof(up_region), &r, sizeof r);
                std::memcpy(h + 8 + ps.target_cap * sizeof(up_region) + d * S * 4, k, S * 4);
            } else if (ps.target) {
                HIPCHK(hipMemcpy(ps.target + 8 + d * sizeof(up_region), &r, sizeof r, hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(ps.target + 8 + ps.target_cap * sizeof(up_region) + d * S * 4, k, S * 4,
                                 hipMemcpyHostToDevice));
            } else {
                c->hp_regions[slot].p[d] = r;
                std::memcpy(c->hp_counts[slot].p + d * S, k, S * 4);
            }
            // (stored scores: only the extent matters) -- async fills, no
            // round trip per record
            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(c->d_q11_st.p + d), r.left, 1, c->stream));
            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(c->d_q11_en.p + d), r.right, 1, c->stream));
            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(c->d_q11_src.p + d), r.unit, 1, c->stream));
            c->q11_rep.push_back({d, soff[i]});
            ++d;
        }
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    c->nreg = total;
    return UP_OK;
}

static int run_replay(up_ctx *c, uint64_t *n_regions);

// threshold <= 0 (q11_mode): one K1q pass; units that process position 1
// (an add at <= bw + 1) add the chains of the exact replay around them
// (q11_finish).  With the -w capture on, the whole-buffer replay instead.
static int run_q11(up_ctx *c, uint64_t *n_regions) {
    HIPCHK(hipSetDevice(c->dev));
    int r = sync_units(c);
    if (r) return r;
    const uint32_t nu = (uint32_t)c->units.size();
    std::vector<uint32_t> f(nu, 0);
    bool any = false;
    if (nu) {
        HIPCHK(c->d_q11_head.ensure(nu));
        HIPCHK(hipMemsetAsync(c->d_q11_head.p, 0, nu * sizeof(uint32_t), c->stream));
        hipLaunchKernelGGL(q11_head_kernel, dim3(nu), dim3(256), 0, c->stream, c->d_units.p,
                           (int)c->p.n_samples, (int)c->p.bw, c->d_q11_head.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(f.data(), c->d_q11_head.p, nu * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (uint32_t v : f) any |= v != 0;
        if (any && (c->prof_capture || q11_whole_replay())) return run_replay(c, n_regions);
        std::vector<int32_t> ub(nu);  // the placement's buffer column
        for (uint32_t i = 0; i < nu; ++i) ub[i] = c->units[i].buffer;
        HIPCHK(c->d_unit_buffer.ensure(nu));
        HIPCHK(hipMemcpy(c->d_unit_buffer.p, ub.data(), nu * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    c->q11_run = true;
    c->q11_place_in_pass = !any;
    r = up_run_async(c);
    if (!r) r = up_run_wait(c, nullptr);
    c->q11_run = false;
    if (r) return r;
    const auto t0 = std::chrono::steady_clock::now();
    if ((r = q11_finish(c, any ? &f : nullptr))) return r;
    c->times[3] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (n_regions) *n_regions = c->nreg;
    return UP_OK;
}

int up_run(up_ctx *c, uint64_t *n_regions) {
    if (!c) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;
    int rc = check_params(c);
    if (rc) return rc;
    if (replay_mode(c)) return run_replay(c, n_regions);
    if (q11_mode(c)) return run_q11(c, n_regions);
    int r = up_run_async(c);
    if (r) return r;
    return up_run_wait(c, n_regions);
}

int up_set_timing(up_ctx *c, int level) {
    if (!c || level < 0 || level > 2) return UP_E_ARG;
    c->timing = level;  // passes already in flight keep the level they were launched with
    return UP_OK;
}

int up_get_regions(up_ctx *c, up_region *out, uint32_t *counts, size_t cap) {
    const up_region *r = nullptr;
    const uint32_t *k = nullptr;
    uint64_t nreg = 0;
    int rc = up_regions_view(c, &r, &k, &nreg);
    if (rc) return rc;
    const size_t n = nreg < cap ? (size_t)nreg : cap;
    if (n && out) std::memcpy(out, r, n * sizeof(up_region));
    if (n && counts) std::memcpy(counts, k, n * c->p.n_samples * sizeof(uint32_t));
    return UP_OK;
}

static void drop_target(up_ctx *c) {
    if (c->target_host && busy(c)) {  // a pass in flight may still write it
        launcher_drain(c);
        sync_all(c);
    }
    if (c->target_host) (void)hipHostUnregister(c->target_host);
    c->target_host = nullptr;
    c->target = nullptr;
    c->target_hostp = nullptr;
    c->target_cap = 0;
}

int up_set_record_target(up_ctx *c, void *buf, uint64_t cap) {
    if (!c || (buf && cap == 0)) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    drop_target(c);
    c->ran = false;
    if (!buf) return UP_OK;
    hipPointerAttribute_t attr{};
    const bool known = hipPointerGetAttributes(&attr, buf) == hipSuccess;
    (void)hipGetLastError();  // an unregistered host pointer reports an error here
    if (known && attr.type == hipMemoryTypeDevice) {
        c->target = (uint8_t *)buf;
    } else {
        // host memory (e.g. a node-shared segment): pin it and let K3 write
        // through the device mapping
        const uint64_t bytes = 8 + cap * (sizeof(up_region) + (uint64_t)c->p.n_samples * sizeof(uint32_t));
        if (!known || attr.type != hipMemoryTypeHost) {
            HIPCHK(hipHostRegister(buf, bytes, hipHostRegisterMapped));
            c->target_host = buf;
        }
        void *dptr = nullptr;
        HIPCHK(hipHostGetDevicePointer(&dptr, buf, 0));
        c->target = (uint8_t *)dptr;
        c->target_hostp = buf;
    }
    c->target_cap = cap;
    return UP_OK;
}

int up_host_register(up_ctx *c, void *ptr, uint64_t bytes) {
    if (!c || !ptr || bytes == 0) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
    c->host_regs.push_back(ptr);
    return UP_OK;
}

int up_regions_view(up_ctx *c, const up_region **regions, const uint32_t **counts, uint64_t *n) {
    if (!c || !regions || !n) return UP_E_ARG;
    if (!c->ran) return UP_E_STATE;
    // the completed pass's own delivery decides (the caller may already have
    // set another target for passes launched after it)
    if (!c->host_regions && c->pass[c->cur_slot].target) return UP_E_STATE;  // records went to the target
    *n = c->nreg;
    if (c->host_regions) {
        *regions = c->h_regions.data();
        if (counts) *counts = c->h_counts.data();
    } else {
        *regions = c->hp_regions[c->cur_slot].p;
        if (counts) *counts = c->hp_counts[c->cur_slot].p;
    }
    return UP_OK;
}

static int shift_run(up_ctx *c, const uint64_t *idx, size_t n, uint16_t max_shift, double *out,
                     uint16_t *best, double *best_corr);

int up_shift_scan(up_ctx *c, const uint64_t *idx, size_t n, uint16_t max_shift, double *out) {
    if (!c || (n && (!idx || !out))) return UP_E_ARG;
    return shift_run(c, idx, n, max_shift, out, nullptr, nullptr);
}

int up_shift_best(up_ctx *c, const uint64_t *idx, size_t n, uint16_t max_shift, uint16_t *best,
                  double *best_corr) {
    if (!c || (n && (!idx || !best || !best_corr))) return UP_E_ARG;
    return shift_run(c, idx, n, max_shift, nullptr, best, best_corr);
}

static int shift_run(up_ctx *c, const uint64_t *idx, size_t n, uint16_t max_shift, double *out,
                     uint16_t *best, double *best_corr) {
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (!c->ran) return UP_E_STATE;
    if (!c->p.nondir) return UP_E_UNSUPPORTED;
    if (n == 0) return UP_OK;
    HIPCHK(hipSetDevice(c->dev));
    up_ctx::Pass &ps = c->pass[c->cur_slot];  // the last completed pass's region lists
    std::vector<uint32_t> st(c->nreg), en(c->nreg);
    std::unordered_map<uint64_t, uint64_t> qrep;  // placed K1q list: its replayed records
    if (c->q11_placed) {
        // K1q records: their stored positions left - 1 .. right - 1 of their
        // source unit, as q11_scatter_kernel wrote them
        for (const auto &e : c->q11_rep) qrep[e.first] = e.second;
        if (c->nreg) {
            HIPCHK(hipMemcpy(st.data(), c->d_q11_st.p, c->nreg * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(en.data(), c->d_q11_en.p, c->nreg * 4, hipMemcpyDeviceToHost));
        }
        HIPCHK(ps.d_starts.ensure(c->nreg + 1));
        HIPCHK(ps.d_ends.ensure(c->nreg + 1));
        HIPCHK(ps.d_runit.ensure(c->nreg + 1));
        HIPCHK(hipMemcpy(ps.d_starts.p, c->d_q11_st.p, c->nreg * 4, hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(ps.d_ends.p, c->d_q11_en.p, c->nreg * 4, hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(ps.d_runit.p, c->d_q11_src.p, c->nreg * 4, hipMemcpyDeviceToDevice));
    } else if (c->host_regions) {
        // replayed (Q1) regions carry state-machine scores the dense KDE
        // cannot reproduce; refuse rather than return something else
        std::vector<uint32_t> un(c->nreg);
        for (uint64_t i = 0; i < c->nreg; ++i) {
            st[i] = c->h_regions[i].left;
            en[i] = c->h_regions[i].right;
            un[i] = c->h_regions[i].unit;
        }
        // replayed regions (Q1 heads, whole-buffer replay) correlate the
        // scores the state machine stored (Region::scores), copied below
        HIPCHK(ps.d_starts.ensure(c->nreg + 1));
        HIPCHK(ps.d_ends.ensure(c->nreg + 1));
        HIPCHK(ps.d_runit.ensure(c->nreg + 1));
        HIPCHK(hipMemcpy(ps.d_starts.p, st.data(), c->nreg * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ps.d_ends.p, en.data(), c->nreg * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(ps.d_runit.p, un.data(), c->nreg * 4, hipMemcpyHostToDevice));
    } else {
        HIPCHK(hipMemcpy(st.data(), ps.d_starts.p, c->nreg * 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(en.data(), ps.d_ends.p, c->nreg * 4, hipMemcpyDeviceToHost));
    }
    // global slab space only for regions whose scores do not stay in K4's
    // LDS: replayed ones (their stored scores are copied in) and long ones
    std::vector<uint64_t> off(n, 0);
    std::vector<uint8_t> pref(n + 1, 0);
    uint64_t tot = 0;
    for (size_t j = 0; j < n; ++j) {
        if (idx[j] >= c->nreg) return UP_E_ARG;
        const uint64_t len = (uint64_t)en[idx[j]] - st[idx[j]] + 1;
        pref[j] = c->q11_placed ? (qrep.count(idx[j]) ? 1 : 0)
                                : (c->host_regions && c->h_emulated[idx[j]] == 1 ? 1 : 0);
        if (pref[j] || len > (uint64_t)kShiftLds) {
            off[j] = tot;
            tot += 2ull * len;
        }
    }
    // table mode: n x (max_shift + 1) correlations; best mode: per region
    // the chosen shift (uint16, packed after the n best correlations)
    const size_t nout = best ? n + (n + 3) / 4 : n * ((size_t)max_shift + 1);
    HIPCHK(c->d_sh_idx.ensure(n));
    HIPCHK(c->d_sh_off.ensure(n));
    HIPCHK(c->d_sh_slab.ensure(tot + 1));
    HIPCHK(c->d_sh_out.ensure(nout));
    HIPCHK(c->d_sh_pref.ensure(n + 1));
    uint64_t *d_idx = c->d_sh_idx.p, *d_off = c->d_sh_off.p;
    double *d_slab = c->d_sh_slab.p, *d_out = c->d_sh_out.p;
    uint8_t *d_pref = c->d_sh_pref.p;
    HIPCHK(hipMemcpyAsync(d_idx, idx, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_off, off.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    for (size_t j = 0; j < n; ++j) {
        if (!pref[j]) continue;
        const uint64_t so = c->q11_placed ? qrep[idx[j]] : c->h_score_off[idx[j]];
        if (so == ~0ull) return UP_E_INTERNAL;
        const uint64_t len = (uint64_t)en[idx[j]] - st[idx[j]] + 1;
        HIPCHK(hipMemcpyAsync(d_slab + off[j], c->d_emu_scores.p + so, 2 * len * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(hipMemcpyAsync(d_pref, pref.data(), n + 1, hipMemcpyHostToDevice, c->stream));
    StatParams P = stat_params(c, ps);
    const size_t lds = kShiftLdsBytes;
    const unsigned blocks = (unsigned)std::min<size_t>(n, 8192);
    {
        const void *k = shift_kernel_for(P.bw, pool_mode(c));
        uint32_t nn = (uint32_t)n;
        int ms = (int)max_shift;
        double *tab = best ? nullptr : d_out;
        uint16_t *bs = best ? (uint16_t *)(d_out + n) : nullptr;
        double *bc = best ? d_out : nullptr;
        void *args[] = {&P, &d_idx, &nn, &ms, &d_off, &d_slab, &d_pref, &tab, &bs, &bc};
        (void)hipLaunchKernel(k, dim3(blocks), dim3(kShiftThreads), args, lds, c->stream);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    if (best) {
        HIPCHK(hipMemcpy(best_corr, d_out, n * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(best, d_out + n, n * 2, hipMemcpyDeviceToHost));
    } else {
        HIPCHK(hipMemcpy(out, d_out, nout * 8, hipMemcpyDeviceToHost));
    }
    return UP_OK;
}

int up_timings(up_ctx *c, double *ms, int n) {
    if (!c || !ms) return UP_E_ARG;
    for (int i = 0; i < n && i < 5; ++i) ms[i] = c->times[i];
    return UP_OK;
}

int up_unit_profile_range(up_ctx *c, uint32_t unit, uint64_t first, uint32_t count, double *out_f,
                          double *out_r) {
    int r = check_runnable(c, true);
    if (r) return r;
    if (busy(c)) return UP_E_STATE;  // a pass in flight reads this state
    if (unit >= c->units.size() || !out_f || first < 1 || count == 0) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    if ((r = sync_units(c))) return r;
    const Unit &u = c->units[unit];
    const uint64_t dom = (uint64_t)u.nstrips * kStrip;  // scan domain incl. Q16 tail
    if (first + count - 1 > dom) return UP_E_ARG;
    double *d = nullptr;
    HIPCHK(hipMalloc(&d, 2 * (size_t)count * sizeof(double) + 16));
    HIPCHK(hipMemsetAsync(d, 0, 2 * (size_t)count * sizeof(double), c->stream));
    ScanParams P = scan_params(c, c->pass[0], c->ovf_cap);  // no pass in flight; records unused
    P.prof_f = d;
    P.prof_r = d + count;
    P.prof_first = (int64_t)first;
    P.prof_len = count;
    P.prof_unit = unit;
    const uint32_t s0 = u.strip0 + (uint32_t)((first - 1) / kStrip);
    const uint32_t s1 = u.strip0 + (uint32_t)((first + count - 2) / kStrip) + 1;
    dispatch_scan<true, kModeFused>(c, c->stream, P, s0, s1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(out_f, d, (size_t)count * sizeof(double), hipMemcpyDeviceToHost));
    if (out_r) HIPCHK(hipMemcpy(out_r, d + count, (size_t)count * sizeof(double), hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return UP_OK;
}

int up_unit_profile(up_ctx *c, uint32_t unit, double *out_f, double *out_r, uint32_t len) {
    if (!out_r) return UP_E_ARG;
    return up_unit_profile_range(c, unit, 1, len, out_f, out_r);
}

// Achievable HBM rate on this device: device-to-device copy of `bytes`
// (read + write), best of `reps`, reported as (2 * bytes) / time.
int up_hbm_copy_gbps(up_ctx *c, uint64_t bytes, int reps, double *gbps) {
    if (!c || !gbps || bytes < 16 || bytes % 16 || reps < 1) return UP_E_ARG;
    HIPCHK(hipSetDevice(c->dev));
    void *a = nullptr, *b = nullptr;
    HIPCHK(hipMalloc(&a, bytes));
    if (hipMalloc(&b, bytes) != hipSuccess) {
        (void)hipFree(a);
        return UP_E_NOMEM;
    }
    HIPCHK(hipMemsetAsync(a, 1, bytes, c->stream));
    float best = 0;
    for (int i = 0; i <= reps; ++i) {
        HIPCHK(hipEventRecord(c->ev[5], c->stream));
        hipLaunchKernelGGL(hbm_copy_kernel, dim3((unsigned)((bytes / 16 + 255) / 256)), dim3(256), 0, c->stream,
                           (const u32x4 *)a, (u32x4 *)b, (uint64_t)(bytes / 16));
        HIPCHK(hipEventRecord(c->ev[6], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[6]));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev[5], c->ev[6]);
        if (i > 0 && (best == 0 || ms < best)) best = ms;  // first copy is a warm-up
    }
    (void)hipFree(a);
    (void)hipFree(b);
    *gbps = 2.0 * (double)bytes / (best * 1e-3) / 1e9;
    return UP_OK;
}


int up_set_profile_capture(up_ctx *c, int on) {
    if (!c) return UP_E_ARG;
    if (busy(c)) return UP_E_STATE;
    c->prof_capture = on != 0;
    return UP_OK;
}

int up_unit_replay_profile(up_ctx *c, uint32_t unit, uint32_t *resync, uint64_t *n, uint32_t *event,
                           uint32_t *pos, double *score, uint64_t cap) {
    if (!c || !resync || !n) return UP_E_ARG;
    if (!c->ran) return UP_E_STATE;
    if (unit >= c->units.size()) return UP_E_ARG;
    *resync = unit < c->h_resync.size() ? c->h_resync[unit] : 0u;
    if (*resync != 0 && !c->prof_capture) return UP_E_STATE;  // replayed without the capture on
    const uint64_t lo = unit + 1 < c->h_pf_off.size() ? c->h_pf_off[unit] : 0;
    const uint64_t hi = unit + 1 < c->h_pf_off.size() ? c->h_pf_off[unit + 1] : 0;
    *n = hi - lo;
    if (!event && !pos && !score) return UP_OK;  // size query
    if (cap < hi - lo || !event || !pos || !score) return UP_E_ARG;
    for (uint64_t i = lo; i < hi; ++i) {
        event[i - lo] = c->h_pf_event[i];
        pos[i - lo] = c->h_pf_pos[i];
        score[i - lo] = c->h_pf_score[i];
    }
    return UP_OK;
}
