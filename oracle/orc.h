/*
 * oracle/orc.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of UniPeak 1.0's KDE smoothing + enriched-region scan, used
 * as the parity checker for the MI355X product path (and as the timed CPU
 * baseline in bench.py).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product (libunipeak_hip.so and the
 * bin/ CLIs) never links or calls it.
 *
 * Parity status: the reference cannot be built in this image (it needs Boost
 * headers/libraries that are absent; writing stand-ins is not allowed), and it
 * ships no tests or fixtures.  This restatement is pinned against the known
 * answers recorded from the reference's own runs in SURVEY.md (see
 * tests/golden/survey_kat.json and tests/test_oracle_kat.py); everything else
 * is "parity partially pinned".
 *
 * Every function cites the reference file:line whose behaviour it restates
 * (paths relative to the reference root).
 */
#ifndef UNIPEAK_ORACLE_H
#define UNIPEAK_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- kernel weights: misc/kernel.cpp:12-35 ---------------------------- */
void orc_kernel(uint16_t bw, double sum, double *w /* 2*bw+1 */);

/* ---- streaming profile buffer: misc/peakcall.cpp:33-231 ---------------- */
typedef struct orc_region orc_region;
typedef struct orc_buf orc_buf;

/* region sink: called when a region passes the filters (peakcall.cpp:45);
 * ownership of the region transfers to the callee (free with
 * orc_region_free). */
typedef void (*orc_region_cb)(void *user, orc_region *r);
/* profile sink: PosScore written when score != 0 (peakcall.cpp:59-62) */
typedef void (*orc_profile_cb)(void *user, int forward, uint32_t contig,
                               uint32_t pos, double score);

orc_buf *orc_buf_new(const double *kernel, uint32_t kernel_size,
                     double region_thr, double kurt_thr, double corr_thr,
                     double hit_thr, int forward, uint16_t n_expt,
                     const uint8_t *control, const double *coeffs,
                     uint32_t n_coeffs, orc_region_cb cb, void *cb_user,
                     orc_profile_cb pcb, void *pcb_user);
void orc_buf_free(orc_buf *b);
/* counts == NULL means an empty HitCountVec (used by flushContig) */
void orc_buf_add(orc_buf *b, const uint32_t *counts, uint32_t contig,
                 uint32_t pos, int forward);
uint64_t orc_buf_flush(orc_buf *b);
uint64_t orc_buf_nregions(const orc_buf *b);
uint64_t orc_buf_nrejects(const orc_buf *b);
const uint64_t *orc_buf_tags_in_regions(const orc_buf *b);

/* ---- region model / statistics: misc/data.cpp:92-193 ------------------ */
int orc_region_forward(const orc_region *r);
uint32_t orc_region_contig(const orc_region *r);
uint32_t orc_region_left(const orc_region *r);
uint32_t orc_region_npos(const orc_region *r);
uint32_t orc_region_peak(const orc_region *r);
double orc_region_peak_score(const orc_region *r);
void orc_region_expt_sums(const orc_region *r, uint32_t *out /* n_expt */);
uint32_t orc_region_sum(const orc_region *r);
double orc_region_kurtosis(const orc_region *r);
double orc_region_corr(const orc_region *r, uint16_t shift);
void orc_region_scores(const orc_region *r, double *f, double *rev);
void orc_region_free(orc_region *r);

/* ---- single-unit convenience for parity tests ------------------------- */
/* Runs one ProfileBuffer over a sparse list of adds of ONE contig and
 * flushes it.  hits: n entries (pos ascending), counts row-major [n][S] for
 * the forward adds, counts_rev likewise for reverse adds (NULL if none).
 * Returns the number of ACCEPTED+REJECTED candidate regions written to out
 * (cap entries), each described by orc_unit_region. */
typedef struct {
    uint32_t left, right, peak, npos, contig;
    int32_t forward, accepted;
    uint32_t sum;
    double peak_score, kurtosis, corr;
} orc_unit_region;

int64_t orc_run_unit(const double *kernel, uint32_t kernel_size,
                     double region_thr, double kurt_thr, double corr_thr,
                     double hit_thr, int buffer_forward, int nondir,
                     uint16_t n_expt, const uint8_t *control,
                     const double *coeffs, uint32_t n_coeffs,
                     uint32_t contig, size_t n, const uint32_t *pos,
                     const uint32_t *counts_fwd, const uint32_t *counts_rev,
                     orc_unit_region *out, uint32_t *out_sums, size_t cap);

/* dense profile of one unit (f and r for positions 1..len) -- computed by
 * running the state machine with a profile sink; positions never processed
 * stay 0. */
int orc_unit_profile(const double *kernel, uint32_t kernel_size,
                     int buffer_forward, int nondir, uint16_t n_expt,
                     const uint8_t *control, const double *coeffs,
                     uint32_t n_coeffs, size_t n, const uint32_t *pos,
                     const uint32_t *counts_fwd, const uint32_t *counts_rev,
                     uint32_t len, double *score_out);

/* ---- CLI restatements (src/regions.cpp, src/strand_shift.cpp,
 *      src/tags_in_regions.cpp) -- main-style entry points ------------- */
int orc_regions_main(int argc, char **argv);
int orc_strand_shift_main(int argc, char **argv);
int orc_tags_in_regions_main(int argc, char **argv);

/* ---- synthetic hg19-shaped generator (bench + tests) ------ */
/* Deterministic counter-based tag counts (spec: DESIGN.md "Synthetic
 * input"); the device generator (unipeak_amd/csrc/synth.hip) follows the
 * same spec.  Writes the nonzero positions (1-based, ascending) of one
 * (sample seed, contig index, strand) track of length len; background tags
 * and peak tags are both confined to [2bw+2, len-2bw-1].  nondir: reverse
 * strand peaks share the forward centres, shifted by +150.  Returns the
 * number of nonzero positions (may exceed cap; only cap are written). */
size_t orc_synth_track(uint64_t seed, uint32_t contig, int strand, int nondir,
                       uint32_t len, uint16_t bw, int with_peaks,
                       uint32_t *pos, uint32_t *cnt, size_t cap);
/* the same track moved by `offset` (the wiggle reader's -s) and, with
 * peak_seed != 0, in replicate mode (shared peak centres) */
size_t orc_synth_track_ex(uint64_t seed, uint32_t contig, int strand, int nondir,
                          uint32_t len, uint16_t bw, int with_peaks, int32_t offset,
                          uint64_t peak_seed, uint32_t *pos, uint32_t *cnt, size_t cap);
/* one unit of a synthetic genome run entirely inside the oracle: the
 * (strand, sample) tracks are generated (orc_synth_track_ex; seeds[s],
 * with_peaks[s], offset[strand]), merged by position and fed to one
 * ProfileBuffer in the reference's order (forward add before reverse add at
 * a position, as orc_run_unit), then flushed.  Output as orc_run_unit. */
int64_t orc_genome_unit(const double *kernel, uint32_t kernel_size, double region_thr,
                        double kurt_thr, double corr_thr, double hit_thr, int buffer_forward,
                        int nondir, uint16_t n_expt, const uint8_t *control,
                        const uint64_t *seeds, const uint8_t *with_peaks, uint64_t peak_seed,
                        const int32_t *offset, uint32_t contig, uint32_t len, uint16_t bw,
                        orc_unit_region *out, uint32_t *out_sums, size_t cap);
/* the Poisson thresholds used by the background draw (6 entries) */
void orc_synth_thresholds(double lambda, uint64_t *thr6);

/* hot-path CPU baseline: drive the directional forward+reverse
 * ProfileBuffers over synthetic tracks (pre-generated per contig, not
 * timed) and time only the add/flush calls. */
int orc_baseline_run(uint32_t n_contigs, const uint32_t *lens, uint64_t seed,
                     uint16_t bw, double region_thr, double kurt_thr,
                     double hit_thr, double background, uint64_t *n_pass,
                     uint64_t *n_reject, double *seconds);

/* one (contig, strand) unit of the same baseline on its own buffer over
 * pre-generated hits (units are independent after a flush; callers run
 * them on several threads) */
int orc_baseline_unit(const uint32_t *pos, const uint32_t *cnt, size_t n, uint32_t contig,
                      int strand, uint16_t bw, double region_thr, double kurt_thr,
                      double hit_thr, double background, uint64_t *n_pass,
                      uint64_t *n_reject);

/* "pos count\n" / "pos -count\n" wiggle lines (out: 24 bytes per pair) */
size_t orc_format_pairs(const uint32_t *pos, const uint32_t *cnt, size_t n, int neg,
                        char *out);

#ifdef __cplusplus
}
#endif
#endif
