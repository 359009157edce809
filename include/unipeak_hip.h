/*
 * include/unipeak_hip.h -- the drop-in C-ABI boundary of unipeak-mi355x.
 *
 * The reference's hot path is an in-process C++ class driven position by
 * position (misc/peakcall.hpp:57-77):
 *
 *   Kernel(bw, 1/background)                         misc/kernel.hpp:16
 *   ProfileBuffer(kernel, r, k, u, t, fwd, control,
 *                 coeffs, contigs, regionsOut, prof) misc/peakcall.hpp:57-69
 *   ProfileBuffer::add(counts, contig, pos, fwd)     misc/peakcall.hpp:76
 *   ProfileBuffer::flushContig()                     misc/peakcall.hpp:75
 *   nRegions()/nRegionRejects()/nTagsInRegions()     misc/peakcall.hpp:71-74
 *   Region::exptSums/posKurtosis/strandCorr          misc/data.hpp:66-72
 *
 * On MI355X the same work is done in batches: every add() that one buffer
 * receives between two flushes (one "unit" = one buffer x one contig pass)
 * is a dense per-position count track resident in HBM, and up_run()
 * performs, for all units at once, what the sequence of add()/flushContig()
 * calls computes: pooled counts, the Epanechnikov KDE, the threshold scan,
 * region segmentation and processRegion()'s statistics and filters.
 * Mapping of entry points to the reference interface:
 *
 *   up_kernel_weights   <- Kernel::Kernel            misc/kernel.cpp:16-35
 *   up_open/up_set_params <- ProfileBuffer ctor      misc/peakcall.cpp:88-135
 *   up_add_unit + up_unit_scatter (or up_unit_pack)
 *                        <- the add() calls of one unit misc/peakcall.cpp:161-222
 *   up_run              <- add()'s window scatter + processPosition +
 *                          processRegion + flushContig  misc/peakcall.cpp:33-86,224-231
 *   up_get_regions      <- regionsOut vector + Region statistics
 *                          misc/peakcall.cpp:45, misc/data.cpp:104-193
 *   up_shift_scan       <- Region::strandCorr(shift) loop src/strand_shift.cpp:205-228
 *
 * Conventions: plain C types only; the caller owns host buffers, the library
 * owns device memory; one context per GPU, driven by one host thread (not
 * re-entrant, like ProfileBuffer).  Every entry point returns UP_OK (0) or a
 * negative UP_E_* code (up_strerror); nothing exits the process.
 */
#ifndef UNIPEAK_HIP_H
#define UNIPEAK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UP_OK 0
#define UP_E_ARG (-1)         /* bad argument */
#define UP_E_HIP (-2)         /* HIP runtime error */
#define UP_E_NOMEM (-3)       /* device allocation failed */
#define UP_E_STATE (-4)       /* call out of order (e.g. no params) */
#define UP_E_UNSUPPORTED (-5) /* configuration outside the GPU path */
#define UP_E_NODEV (-6)       /* no HIP device */
#define UP_E_INTERNAL (-7)    /* internal consistency check failed */

typedef struct up_ctx up_ctx;

/* Parameters of one ProfileBuffer pair (misc/peakcall.hpp:57-69) as the
 * CLI computes them (src/regions.cpp:152-232, src/strand_shift.cpp:131-142). */
typedef struct {
    uint16_t bw;              /* kernel bandwidth (-b) */
    uint16_t n_samples;       /* S = all samples, controls included */
    int32_t nondir;           /* 0: one strand per unit; 1: both strands in one unit */
    double background;        /* kernel sums to 1/background */
    double region_thr;        /* -r */
    double kurt_thr;          /* -k (0 disables) */
    double corr_thr;          /* -u (<= -1 disables) */
    double hit_thr;           /* already multiplied by S_nc where the CLI does */
    const uint8_t *is_control;/* [S] or NULL */
    const double *coeffs;     /* NULL or [n_coeffs] = normalised -z coefficients */
    uint32_t n_coeffs;
    int32_t want_corr;        /* evaluate strandCorr(0) for every region */
} up_params;

#define UP_CLOSE_RULE 0xFFFFFFFFu
/* region threshold <= 0 (quirk Q11, run in parallel): closed by the add
 * after the unit's first add at pos >= right + bw + 1 (the first add at a
 * larger position), else by the unit's flush */
#define UP_CLOSE_Q11 0xFFFFFFFEu
/* region threshold <= 0: the region the buffer's previous unit left open
 * after its flush, relabelled to this unit (misc/peakcall.cpp:164-168) and
 * closed by this unit's first add at a position above its first add's, else
 * by its flush; left/right/peak are positions of the previous unit */
#define UP_CLOSE_Q11_HEAD 0xFFFFFFFDu

/* One candidate region (accepted or rejected by processRegion). */
typedef struct {
    uint32_t unit;            /* unit the region was closed in */
    uint32_t left, right;     /* inclusive positions (right may exceed the contig, Q16) */
    uint32_t peak;            /* first position of the maximal f+r */
    uint32_t sum;             /* Region::sum() (uint32, wraps) */
    uint32_t nonctl_sum;      /* sum over non-control samples of exptSums */
    int32_t accepted;         /* passed the hit/kurtosis/correlation filters */
    uint32_t close_pos;       /* UP_CLOSE_RULE: closed by the unit's first add at
                                 pos >= right + bw + 2, else by its flush;
                                 UP_CLOSE_Q11 / UP_CLOSE_Q11_HEAD: threshold
                                 <= 0, see above;
                                 0: closed by the unit's flush; otherwise the
                                 position of the add whose retirement closed it
                                 (head-hit units replayed by the emulator, Q1) */
    double peak_score;        /* f+r at peak */
    double kurtosis;          /* Region::posKurtosis() */
    double corr;              /* Region::strandCorr(0) or NaN when not evaluated */
} up_region;

/* library / device */
int up_version(void);
/* bits per stored count in a device track: the K1a stream
 * reads bits/8 bytes per position per strand per non-control sample */
int up_track_bits(void);
const char *up_strerror(int code);
int up_device_count(int *n);

/* Kernel::Kernel(bw, sum) -- 2*bw+1 weights into w (host computation). */
int up_kernel_weights(uint16_t bw, double sum, double *w);

int up_open(int hip_device, up_ctx **out);
void up_close(up_ctx *ctx);
int up_set_params(up_ctx *ctx, const up_params *p);

/* Units.  A unit is one ProfileBuffer (buffer_id 0 = forward buffer, 1 =
 * reverse buffer) over one contig pass; units of one buffer must be added in
 * the order the buffer sees them.  nstrands is 1 (directional) or 2
 * (nondirectional: strand 0 forward, 1 reverse).  Tracks start zeroed and
 * cover positions 1..contig_len; in device memory they are up_track_bits()-bit
 * counts (2: four positions per byte) whose largest value is an escape into
 * an exact per-unit overflow table, so any uint32 count can
 * be written.
 * Quirk Q1 (misc/peakcall.cpp:177-183): a unit with pooled tags at a position
 * <= bw is replayed by the exact state machine; if all of its adds sit at
 * positions <= bw its leftover state leaks into the buffer's NEXT unit, which
 * must then be in the same context (the reference driver's chain). */
int up_add_unit(up_ctx *ctx, uint32_t contig_len, int32_t nstrands,
                int32_t buffer_id, uint32_t *unit_id);
int up_unit_count(up_ctx *ctx, uint32_t *n);
/* replace a track from DEVICE-resident dense uint32 counts: position p
 * (1-based) at dev_counts[p-1], contig_len elements (same device) */
int up_unit_pack(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                 const uint32_t *dev_counts);
/* write n (pos, count) host pairs into a track: positions 1..len, each at
 * most once per call (UP_E_ARG otherwise: one nibble written twice would OR
 * two counts together); a count of 0 clears the position */
int up_unit_scatter(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                    size_t n, const uint32_t *pos, const uint32_t *counts);
/* fill a track with the synthetic hg19-shaped spec */
int up_unit_synth(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                  uint64_t seed, uint32_t contig_index, int32_t synth_strand,
                  int32_t nondir, int32_t with_peaks);
/* the same track moved by `offset` positions, as the wiggle reader's -s
 * shift moves it (forward strand +s, reverse -s, misc/format.cpp:693-705):
 * position p holds the spec's count at p - offset; counts that leave
 * [1, contig_len] are dropped */
int up_unit_synth_offset(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                         uint64_t seed, uint32_t contig_index, int32_t synth_strand,
                         int32_t nondir, int32_t with_peaks, int32_t offset);
/* the same with peak_seed != 0: replicate samples -- peak
 * centres drawn from peak_seed and shared by every sample generated with it,
 * per-sample heights, centre jitter (-20..+20) and tag offsets from `seed`;
 * peak_seed 0 is up_unit_synth_offset */
int up_unit_synth_ex(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                     uint64_t seed, uint32_t contig_index, int32_t synth_strand,
                     int32_t nondir, int32_t with_peaks, int32_t offset, uint64_t peak_seed);
/* total tags of one track (sum of its counts, uint64) */
int up_unit_tag_total(up_ctx *ctx, uint32_t unit, int32_t strand, uint16_t sample,
                      uint64_t *total);
/* override the last add position of a unit (host knows control-only adds) */
int up_unit_set_last_add(up_ctx *ctx, uint32_t unit, uint32_t last_add);
int up_unit_last_add(up_ctx *ctx, uint32_t unit, uint32_t *last_add);
int up_reset_units(up_ctx *ctx);

/* Run K1..K3 over every unit (stream-ordered, blocking).  A region
 * threshold <= 0 makes the leap branch of processPosition live (quirk Q11):
 * with non-negative scores every run of processed positions is a region,
 * found in parallel (K1q; records as UP_CLOSE_Q11 / UP_CLOSE_Q11_HEAD
 * describe).  A unit that processes position 1 (an add at <= bw + 1) adds a
 * short exact replay (K0) around it, from the start of the buffer's
 * previous unit's last run to the first clean leap past it; those records
 * name their closing add in close_pos like the whole-buffer replay's.
 * bw > UP_MAX_PARALLEL_BW (511: K1's register-resident halo of NH <= 8
 * 64-position words) on directional units with a threshold > 0 runs K1w,
 * the parallel scan for wide kernels (up to 32767, a window of 65535 cells;
 * pipelined like K1; no dense profile).  Wider kernels (32768..65535, where
 * the reference's UShort retirement count wraps, misc/peakcall.cpp:172-177)
 * take the whole-buffer replay.  A negative coefficient at a threshold <= 0, the -w
 * capture with a head unit or with bw > 511, and bw > 511 on nondirectional
 * units or at a threshold <= 0 run the exact state machine over every unit
 * instead (K0, as independent chains from every run start: exact, far
 * slower than the scans); up_run_async refuses those (UP_E_UNSUPPORTED),
 * up_unit_profile* refuse them and bw > 511.  up_shift_scan correlates a
 * replayed region's stored scores (Region::scores), as strandCorr does.
 * With a threshold <= 0 the last region of a unit is still open after its
 * flush and is closed in the buffer's next unit (UP_CLOSE_Q11_HEAD); the
 * last region of a buffer's last unit in the context is never closed (the
 * reference never writes it).  So every unit of one buffer must be in ONE
 * context at -r <= 0: a caller that splits a buffer's units over contexts
 * or ranks loses the region that crosses the split (bin/regions' multi-device
 * split keeps buffers whole for this reason). */
#define UP_MAX_PARALLEL_BW 511
int up_run(up_ctx *ctx, uint64_t *n_regions);
/* Pipelined form of up_run: up_run_async enqueues one pass and returns
 * (at most UP_MAX_IN_FLIGHT passes in flight); up_run_wait completes the OLDEST pass in
 * flight and makes its records current (as up_run would).  Passes in flight
 * overlap on the device: a pass's streaming K1a starts when the previous
 * pass's K1a has ended, beside that pass's exact/segmentation/statistics
 * kernels.  Each pass delivers into the record target that was set when it
 * was launched, so a caller rotates targets; with host delivery the view of
 * a pass stays valid until the UP_MAX_IN_FLIGHT-th following launch.  Units and
 * parameters cannot change while a pass is in flight (UP_E_STATE).  The HIP
 * calls of an async pass run on the context's own launcher thread
 * (UNIPEAK_LAUNCHER=0: on the caller's); a launch failure is returned by the
 * up_run_wait of that pass.  The context is still driven by one caller thread. */
#define UP_MAX_IN_FLIGHT 5
int up_run_async(up_ctx *ctx);
int up_run_wait(up_ctx *ctx, uint64_t *n_regions);
/* device timing of passes launched from now on (passes in flight keep
 * theirs): 0 = wall time only, 1 = + K1a (HIP events around the streaming
 * kernel), 2 = every phase (default).  Each event pair costs a few
 * microseconds of idle GPU between kernels. */
int up_set_timing(up_ctx *ctx, int level);
/* Copy region records (unit-major, left-ascending) and optionally the
 * per-sample exptSums [n][S]. */
int up_get_regions(up_ctx *ctx, up_region *out, uint32_t *counts, size_t cap);
/* Zero-copy view of the same records: host memory owned by the context
 * (pinned), valid until the next up_run / up_reset_units / up_close. */
int up_regions_view(up_ctx *ctx, const up_region **regions, const uint32_t **counts,
                    uint64_t *n);

/* Multi-GPU delivery: make up_run write the records into a caller-owned
 * buffer laid out as
 *   [uint64 n][cap x up_region][cap x n_samples x uint32 exptSums]
 * either DEVICE memory of this context's GPU (hand it to RCCL without a host
 * round trip) or HOST memory, e.g. a node-shared segment rank 0 reads
 * directly (the library pins it and K3 writes through the mapping).
 * up_run fails with UP_E_NOMEM if a pass yields more than cap records.
 * buf = NULL restores host delivery (up_get_regions / up_regions_view). */
int up_set_record_target(up_ctx *ctx, void *buf, uint64_t cap);
/* pin + map a host range once (e.g. every record slot of a node-shared
 * segment), so switching record targets inside it costs nothing; released
 * by up_close */
int up_host_register(up_ctx *ctx, void *ptr, uint64_t bytes);

/* strandCorr(shift) for shift = 0..max_shift of the given regions
 * (indices into up_get_regions order); out is [n][max_shift+1]. */
int up_shift_scan(up_ctx *ctx, const uint64_t *region_idx, size_t n,
                  uint16_t max_shift, double *out);
/* the same regions reduced on the device to strand_shift's per-region
 * choice (src/strand_shift.cpp:209-217): best_shift = the first shift whose
 * strandCorr is the largest value above -1 (0 if none), best_corr = that
 * value (-1 if none) */
int up_shift_best(up_ctx *ctx, const uint64_t *region_idx, size_t n,
                  uint16_t max_shift, uint16_t *best_shift, double *best_corr);

/* The per-dataset index (DESIGN.md §3 "Index policy"): data derived from
 * the packed tracks that repeated passes over the same tracks may reuse --
 * per track a chunk-sum plane (1 byte per 16 positions), per unit a pooled
 * plane and, with several pooled samples, a pooled count track (1 byte per
 * position and strand).  The reference makes ONE pass per run
 * (src/regions.cpp:311-391): a pass without the index reads only the packed
 * tracks and pays no build.  Policies:
 *   UP_INDEX_AUTO   (default) the first pass after a track or pooling change
 *                   runs without it; the index is built (one launch per
 *                   kind over every stale unit) before the second;
 *   UP_INDEX_NEVER  no pass uses it: every pass costs what one cold pass
 *                   costs (bw > UP_MAX_PARALLEL_BW still builds it: K1w
 *                   screens on the planes);
 *   UP_INDEX_ALWAYS built before the first pass.
 * Refused while a pass is in flight (UP_E_STATE).  up_invalidate_index drops
 * what was built (the next pass that wants it rebuilds it; AUTO counts
 * passes anew).  up_index_state: *on = the next pass uses the index now,
 * *builds = index builds so far in this context. */
#define UP_INDEX_AUTO 0
#define UP_INDEX_NEVER 1
#define UP_INDEX_ALWAYS 2
int up_set_index_policy(up_ctx *ctx, int policy);
int up_invalidate_index(up_ctx *ctx);
int up_index_state(up_ctx *ctx, int *on, uint64_t *builds);
/* bytes the streaming scan (K1a) reads per 1,024 positions of a unit in the
 * index state of the moment (its algorithmic bytes): 64 when
 * it streams a chunk-sum plane (index on and bw <= 255: the pooled track's
 * own plane, or the unit's pooled plane of several samples / both strands),
 * else 1024 * up_track_bits() / 8 per pooled track and strand */
int up_scan_density(up_ctx *ctx, uint32_t *bytes_per_1024);
/* device-side timings of the last up_run in ms: [0]=K1 scan, [1]=K2
 * segment, [2]=K3 stats, [3]=whole up_run wall, [4]=K1 launches */
/* achievable HBM rate: a float4 streaming copy kernel of `bytes` (a multiple
 * of 16; best of reps),
 * GB/s counting read + write (the bench's copy-rate reference) */
int up_hbm_copy_gbps(up_ctx *ctx, uint64_t bytes, int reps, double *gbps);
int up_timings(up_ctx *ctx, double *ms, int n);
/* dense per-position score f+r of one unit (testing/-w): out[len] */
int up_unit_profile(up_ctx *ctx, uint32_t unit, double *out_f, double *out_r,
                    uint32_t len);
/* -w for units the exact replay produced (K0: quirk Q1 head hits, -r <= 0
 * with a unit processing position 1 or a negative coefficient,
 * bw > UP_MAX_PARALLEL_BW), whose retirements the dense KDE does not reproduce.  With the
 * capture on before up_run, the replay records every processPosition() with
 * a nonzero score (misc/peakcall.cpp:80-83: profileOut_->write), and
 * up_unit_replay_profile returns them for one unit in emission order:
 * event[i] = index of the unit's add() whose retirement loop wrote it
 * (UP_FLUSH_EVENT: the unit's flushContig()), pos[i], score[i] = f + r.
 * resync = 0: the unit was not replayed (up_unit_profile_range gives its
 * profile); X: the entries cover positions < X and the dense KDE the rest;
 * UP_FLUSH_EVENT (0xFFFFFFFF): the whole unit was replayed.  Call with
 * event/pos/score NULL to get n. */
#define UP_FLUSH_EVENT 0xFFFFFFFFu
int up_set_profile_capture(up_ctx *ctx, int on);
int up_unit_replay_profile(up_ctx *ctx, uint32_t unit, uint32_t *resync, uint64_t *n,
                           uint32_t *event, uint32_t *pos, double *score, uint64_t cap);
/* the same for positions [first, first + count) (first >= 1; the range may
 * run past the contig end into the scan domain, quirk Q16); out_r may be
 * NULL for directional units */
int up_unit_profile_range(up_ctx *ctx, uint32_t unit, uint64_t first, uint32_t count,
                          double *out_f, double *out_r);

/* ---- tags_in_regions (src/tags_in_regions.cpp:131-199) on the GPU ---------
 * A stream is one sample's alignment records in the order the reference's
 * readAlign() returns them (ParseAlignStream / NondirParseAlignStream,
 * misc/format.cpp:503-565, 873-895): key[i] = contig << 32 | firstPos,
 * count[i] (> 0), forward[i].  The reference walks one cursor per stream
 * through the regions (skip to the region's strand at (contig, left), then
 * count every record on the contig at firstPos <= right, any strand: quirk
 * Q12).  up_tir_query answers every (region, stream) pair as if that
 * stream's cursor started at its first record: first = the record the skip
 * loop stops at, end = the record the count loop stops at (n: exhausted),
 * hits = sum of counts in [first, end) (uint32, wrapping like HitCount).
 * That is the reference's answer whenever the real cursor has not passed
 * `first` (nothing in between qualifies); the caller walks the other regions
 * itself (bin/tags_in_regions does).  UP_TIR_HOST in first/end:
 * the query crossed more unsorted runs of the stream than the device walks
 * (an unsorted stream); the caller walks that pair. */
#define UP_TIR_HOST 0xFFFFFFFFu
typedef struct up_tir up_tir;
int up_tir_open(int hip_device, up_tir **out);
void up_tir_close(up_tir *h);
/* upload stream `stream` (0..4095) and build its prefix sums and skip tables
 * on the device (blocking; the host arrays may be freed afterwards) */
int up_tir_set_stream(up_tir *h, uint32_t stream, uint64_t n, const uint64_t *key,
                      const uint32_t *count, const uint8_t *forward);
/* regions r = 0..n_regions-1 against streams 0..n_streams-1; outputs are
 * [n_regions][n_streams] */
int up_tir_query(up_tir *h, uint32_t n_streams, uint64_t n_regions, const uint32_t *contig,
                 const uint32_t *left, const uint32_t *right, const uint8_t *forward,
                 uint32_t *first, uint32_t *end, uint32_t *hits);
/* device time in ms: [0] the last up_tir_set_stream's table build (after the
 * upload), [1] the last up_tir_query's kernel */
int up_tir_timings(up_tir *h, double *ms, int n);

/* ---- convert_align's CountMap (misc/data.cpp:263-314, 321-596) on the GPU --
 * Per (strand, contig) position -> count, as dense uint32 tracks in HBM
 * (2 x the table's total length x 4 B).  up_cm_add = CountMap::add for n
 * alignments (contig < n_contigs, 1 <= pos <= its length, else UP_E_ARG;
 * count NULL = 1 each; per-position counts wrap at 2^32 like HitCount).
 * up_cm_collect = the nonzero entries in the order convert_align writes
 * them: nondir 0 -- CountMap::ConstIterator, forward strand then reverse,
 * contigs in table order, positions ascending; nondir 1 --
 * ConstNondirIterator, both strands merged by position with their counts
 * added (forward[] = 1).  With every output NULL only *n is set; cap is the
 * output arrays' length. */
typedef struct up_cm up_cm;
int up_cm_open(int hip_device, uint32_t n_contigs, const uint32_t *contig_len, up_cm **out);
void up_cm_close(up_cm *h);
int up_cm_add(up_cm *h, uint64_t n, const uint32_t *contig, const uint32_t *pos,
              const uint8_t *forward, const uint32_t *count);
int up_cm_collect(up_cm *h, int nondir, uint64_t *n, uint32_t *contig, uint32_t *pos,
                  uint32_t *count, uint8_t *forward, uint64_t cap);
/* device time in ms: [0] every up_cm_add kernel so far, [1] the last collect */
int up_cm_timings(up_cm *h, double *ms, int n);

#ifdef __cplusplus
}
#endif
#endif
