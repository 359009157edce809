/*
 * oracle/orc_core.c -- TEST INFRASTRUCTURE ONLY (see orc.h header).
 *
 * A plain-C restatement of the reference's streaming smoother/segmenter:
 * the Epanechnikov kernel (misc/kernel.cpp), the ProfileBuffer state
 * machine (misc/peakcall.cpp) and the Region statistics (misc/data.cpp).
 * The window is a fixed ring instead of a deque; otherwise every arithmetic
 * step happens in the reference's order so FP64 results are bit-identical
 * (build with -ffp-contract=off, no -ffast-math).
 *
 * Build flags of the reference (config.mk:2: g++ -ansi -O4) matter here:
 * under C++98 libstdc++'s std::pow(double,int) is __builtin_powi, so
 * pow(d,2) is d*d and pow(d,4) is (d*d)*(d*d).  We restate that directly.
 */
#include "orc.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void die(const char *msg) {
    fprintf(stderr, "oracle: %s\n", msg);
    abort();
}

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) die("out of memory");
    return p;
}

/* ---------------------------------------------------------------------- */
/* misc/kernel.cpp:12-14 (f) and :16-35 (ctor)                             */
/* ---------------------------------------------------------------------- */
void orc_kernel(uint16_t bw, double sum_target, double *w) {
    const int n = 2 * (int)bw + 1;
    double acc = 0;
    for (int i = -(int)bw, j = 0; i <= (int)bw; ++i, ++j) {
        const double x = (double)i / (double)bw;
        /* 3 * (1 - pow(x, 2)) / 4, with pow(x,2) == x*x (powi) */
        w[j] = 3 * (1 - x * x) / 4;
        acc += w[j];
    }
    const double scale = sum_target / acc;
    for (int j = 0; j < n; ++j) w[j] *= scale;
}

/* ---------------------------------------------------------------------- */
/* Region -- misc/data.hpp:54-73, misc/data.cpp:79-193                     */
/* ---------------------------------------------------------------------- */
struct orc_region {
    int forward;
    uint32_t contig;
    uint32_t left;
    uint32_t peak_pos;
    double peak_score;
    uint16_t n_expt;
    uint32_t n, cap;
    uint32_t **hits; /* per position: NULL or n_expt counts */
    double *f, *r;
};

static orc_region *region_new(int forward, uint32_t contig, uint32_t left,
                              uint16_t n_expt) {
    orc_region *g = (orc_region *)xmalloc(sizeof *g);
    memset(g, 0, sizeof *g);
    g->forward = forward;
    g->contig = contig;
    g->left = left;
    g->n_expt = n_expt;
    return g;
}

void orc_region_free(orc_region *g) {
    if (!g) return;
    for (uint32_t i = 0; i < g->n; ++i) free(g->hits[i]);
    free(g->hits);
    free(g->f);
    free(g->r);
    free(g);
}

/* Region::addPos, data.cpp:92-102 */
static void region_add_pos(orc_region *g, uint32_t *hits, double f, double r) {
    if (g->n == g->cap) {
        g->cap = g->cap ? 2 * g->cap : 64;
        g->hits = (uint32_t **)realloc(g->hits, g->cap * sizeof(uint32_t *));
        g->f = (double *)realloc(g->f, g->cap * sizeof(double));
        g->r = (double *)realloc(g->r, g->cap * sizeof(double));
        if (!g->hits || !g->f || !g->r) die("out of memory");
    }
    g->hits[g->n] = hits;
    g->f[g->n] = f;
    g->r[g->n] = r;
    g->n++;
    const double score = f + r;
    if (g->peak_pos == 0 || score > g->peak_score) {
        g->peak_pos = (uint32_t)(g->left + g->n - 1); /* Pos truncation */
        g->peak_score = score;
    }
}

int orc_region_forward(const orc_region *g) { return g->forward; }
uint32_t orc_region_contig(const orc_region *g) { return g->contig; }
uint32_t orc_region_left(const orc_region *g) { return g->left; }
uint32_t orc_region_npos(const orc_region *g) { return g->n; }
uint32_t orc_region_peak(const orc_region *g) { return g->peak_pos; }
double orc_region_peak_score(const orc_region *g) { return g->peak_score; }

void orc_region_scores(const orc_region *g, double *f, double *r) {
    memcpy(f, g->f, g->n * sizeof(double));
    memcpy(r, g->r, g->n * sizeof(double));
}

/* Region::exptSums, data.cpp:116-131 (HitCount = uint32, wraps) */
void orc_region_expt_sums(const orc_region *g, uint32_t *out) {
    for (uint16_t s = 0; s < g->n_expt; ++s) out[s] = 0;
    for (uint32_t i = 0; i < g->n; ++i)
        if (g->hits[i])
            for (uint16_t s = 0; s < g->n_expt; ++s) out[s] += g->hits[i][s];
}

/* Region::sum, data.cpp:104-114 */
uint32_t orc_region_sum(const orc_region *g) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < g->n; ++i)
        if (g->hits[i])
            for (uint16_t s = 0; s < g->n_expt; ++s) acc += g->hits[i][s];
    return acc;
}

static uint32_t pos_count(const orc_region *g, uint32_t i) {
    uint32_t pc = 0;
    for (uint16_t s = 0; s < g->n_expt; ++s) pc += g->hits[i][s];
    return pc;
}

/* Region::posMean, data.cpp:133-148: UShort position index, uint32 sums */
static double region_pos_mean(const orc_region *g) {
    uint32_t count = 0, sum = 0;
    uint16_t pos = 0;
    for (uint32_t i = 0; i < g->n; ++i, ++pos) {
        if (g->hits[i]) {
            const uint32_t pc = pos_count(g, i);
            count += pc;
            sum += pc * (uint32_t)pos;
        }
    }
    return (double)sum / (double)count;
}

/* Region::posKurtosis, data.cpp:164-182 */
double orc_region_kurtosis(const orc_region *g) {
    if (g->n == 0) die("kurtosis of empty region");
    const double x_bar = region_pos_mean(g);
    uint32_t count = 0;
    double sum2 = 0, sum4 = 0;
    uint16_t pos = 0;
    for (uint32_t i = 0; i < g->n; ++i, ++pos) {
        if (g->hits[i]) {
            const uint32_t pc = pos_count(g, i);
            count += pc;
            const double d = (double)pos - x_bar;
            const double d2 = d * d;
            sum2 += (double)pc * d2;
            sum4 += (double)pc * (d2 * d2);
        }
    }
    return ((double)count - 1) * sum4 / (sum2 * sum2);
}

/* mean/sd/corr, data.cpp:22-58 */
static double vmean(const double *a, size_t n) {
    double s = 0;
    for (size_t i = 0; i < n; ++i) s += a[i];
    return s / (double)n;
}
static double vsd(const double *a, size_t n, double m) {
    double ssr = 0;
    for (size_t i = 0; i < n; ++i) {
        const double d = a[i] - m;
        ssr += d * d;
    }
    return sqrt(ssr / ((double)n - 1));
}
static double vcorr(const double *a, const double *b, size_t n) {
    const double m1 = vmean(a, n), m2 = vmean(b, n);
    const double s1 = vsd(a, n, m1), s2 = vsd(b, n, m2);
    double ssr = 0;
    for (size_t i = 0; i < n; ++i) ssr += (a[i] - m1) * (b[i] - m2);
    return ssr / (((double)n - 1) * s1 * s2);
}

/* Region::strandCorr, data.cpp:184-193 */
double orc_region_corr(const orc_region *g, uint16_t shift) {
    if (g->n > (unsigned)(2 * shift + 3)) {
        const size_t n = g->n - 2 * (size_t)shift;
        return vcorr(g->f, g->r + 2 * (size_t)shift, n);
    }
    return NAN; /* numeric_limits<double>::quiet_NaN(): +nan */
}

/* ---------------------------------------------------------------------- */
/* ProfileBuffer -- misc/peakcall.hpp:18-77, misc/peakcall.cpp:33-231       */
/* ---------------------------------------------------------------------- */
typedef struct {
    uint32_t *hits;
    double f, r;
} cell;

struct orc_buf {
    cell *ring; /* window of kernel_size cells, ring[(head+j)%W] = deque[j] */
    uint32_t W, head;
    uint16_t bw;
    const double *kernel;
    orc_region *region;
    double region_thr, kurt_thr, corr_thr, hit_thr;
    int forward;
    uint32_t contig, buffer_pos, last_pos;
    uint64_t n_regions, n_rejects, n_contig_regions;
    uint64_t *tags_in_regions;
    uint8_t *control;
    double *coeffs;
    uint32_t n_coeffs;
    uint16_t n_expt;
    orc_region_cb cb;
    void *cb_user;
    orc_region_cb rej_cb; /* test hook: rejected candidates */
    orc_profile_cb pcb;
    void *pcb_user;
};

static cell *at(orc_buf *b, uint32_t j) { return &b->ring[(b->head + j) % b->W]; }

/* ProfileBuffer::processRegion, peakcall.cpp:33-53 */
static void process_region(orc_buf *b) {
    orc_region *g = b->region;
    uint32_t *sums = (uint32_t *)xmalloc(b->n_expt * sizeof(uint32_t));
    orc_region_expt_sums(g, sums);
    uint32_t non_control = 0;
    for (uint16_t s = 0; s < b->n_expt; ++s)
        if (!b->control[s]) non_control += sums[s];
    int ok = (double)non_control >= b->hit_thr;
    if (ok)
        ok = (b->kurt_thr == 0 ||
              (g->n > 1 && orc_region_kurtosis(g) <= b->kurt_thr));
    if (ok) ok = (b->corr_thr <= -1 || orc_region_corr(g, 0) >= b->corr_thr);
    if (ok) {
        for (uint16_t s = 0; s < b->n_expt; ++s) b->tags_in_regions[s] += sums[s];
        b->n_regions++;
        b->n_contig_regions++;
        if (b->cb) b->cb(b->cb_user, g); else orc_region_free(g);
    } else {
        if (b->rej_cb) b->rej_cb(b->cb_user, g); else orc_region_free(g);
        b->n_rejects++;
    }
    free(sums);
    b->region = region_new(b->forward, b->contig, 0, b->n_expt);
}

/* ProfileBuffer::processPosition, peakcall.cpp:55-86 */
static void process_position(orc_buf *b, uint32_t pos, double f, double r,
                             uint32_t *hits) {
    if (!(pos > b->last_pos)) die("processPosition: pos <= lastPos");
    const double score = f + r;
    orc_region *g = b->region;
    if (pos == b->last_pos + 1) {
        if (g->left != 0) {
            if (score >= b->region_thr) {
                region_add_pos(g, hits, f, r);
            } else {
                process_region(b);
                free(hits);
            }
        } else {
            if (score >= b->region_thr) {
                g->left = pos;
                region_add_pos(g, hits, f, r);
            } else {
                free(hits);
            }
        }
    } else { /* leap */
        if (g->left != 0) process_region(b);
        if (score >= b->region_thr) region_add_pos(b->region, hits, f, r);
        else free(hits);
    }
    if (score != 0 && b->pcb) b->pcb(b->pcb_user, b->forward, b->contig, pos, score);
    b->last_pos = pos;
}

/* ctor, peakcall.cpp:88-135 */
orc_buf *orc_buf_new(const double *kernel, uint32_t kernel_size,
                     double region_thr, double kurt_thr, double corr_thr,
                     double hit_thr, int forward, uint16_t n_expt,
                     const uint8_t *control, const double *coeffs,
                     uint32_t n_coeffs, orc_region_cb cb, void *cb_user,
                     orc_profile_cb pcb, void *pcb_user) {
    if (!(kernel_size > 0 && kernel_size % 2 == 1)) die("kernel size must be odd");
    orc_buf *b = (orc_buf *)xmalloc(sizeof *b);
    memset(b, 0, sizeof *b);
    b->W = kernel_size;
    b->ring = (cell *)xmalloc(kernel_size * sizeof(cell));
    memset(b->ring, 0, kernel_size * sizeof(cell));
    b->bw = (uint16_t)((kernel_size - 1) / 2);
    b->kernel = kernel;
    b->region = region_new(1, 0, 0, n_expt); /* Q2: first region is forward */
    b->region_thr = region_thr;
    b->kurt_thr = kurt_thr;
    b->corr_thr = corr_thr;
    b->hit_thr = hit_thr;
    b->forward = forward;
    b->n_expt = n_expt;
    b->tags_in_regions = (uint64_t *)xmalloc(n_expt * sizeof(uint64_t));
    memset(b->tags_in_regions, 0, n_expt * sizeof(uint64_t));
    b->control = (uint8_t *)xmalloc(n_expt);
    uint16_t n_control = 0;
    for (uint16_t s = 0; s < n_expt; ++s) {
        b->control[s] = control ? (control[s] != 0) : 0;
        n_control += b->control[s];
    }
    b->n_coeffs = n_coeffs;
    b->coeffs = (double *)xmalloc((n_coeffs ? n_coeffs : 1) * sizeof(double));
    if (n_coeffs) memcpy(b->coeffs, coeffs, n_coeffs * sizeof(double));
    if (!(n_coeffs == 0 || n_control + n_coeffs == n_expt))
        die("coefficient count mismatch");
    b->cb = cb;
    b->cb_user = cb_user;
    b->pcb = pcb;
    b->pcb_user = pcb_user;
    return b;
}

void orc_buf_free(orc_buf *b) {
    if (!b) return;
    for (uint32_t j = 0; j < b->W; ++j) free(b->ring[j].hits);
    free(b->ring);
    orc_region_free(b->region);
    free(b->tags_in_regions);
    free(b->control);
    free(b->coeffs);
    free(b);
}

uint64_t orc_buf_nregions(const orc_buf *b) { return b->n_regions; }
uint64_t orc_buf_nrejects(const orc_buf *b) { return b->n_rejects; }
const uint64_t *orc_buf_tags_in_regions(const orc_buf *b) { return b->tags_in_regions; }

/* ProfileBuffer::add, peakcall.cpp:161-222 */
void orc_buf_add(orc_buf *b, const uint32_t *counts, uint32_t contig,
                 uint32_t pos, int forward) {
    if (contig != b->contig) {
        orc_buf_flush(b);
        b->contig = contig;
        b->region->contig = contig;
    }
    if (!(pos >= b->buffer_pos)) die("add: positions out of order");
    uint16_t n_static = (uint16_t)b->W;
    if (pos <= b->buffer_pos + 2u * b->bw) n_static = (uint16_t)(pos - b->buffer_pos);
    if (b->buffer_pos != 0) {
        for (uint16_t i = 0; i < n_static; ++i) {
            if (b->buffer_pos + i > b->bw) {
                cell *front = at(b, 0);
                uint32_t *h = front->hits;
                const double f = front->f, r = front->r;
                front->hits = NULL; /* ownership moves to processPosition */
                process_position(b, b->buffer_pos + i - b->bw, f, r, h);
                /* pop_front + push_back(BufferPos()) */
                front->f = 0;
                front->r = 0;
                b->head = (b->head + 1) % b->W;
            }
        }
    }
    double count_sum = 0;
    if (counts) {
        if (b->n_coeffs == 0) {
            for (uint16_t s = 0; s < b->n_expt; ++s)
                if (!b->control[s]) count_sum += (double)counts[s];
        } else {
            uint32_t k = 0;
            for (uint16_t s = 0; s < b->n_expt && k < b->n_coeffs; ++s)
                if (!b->control[s]) {
                    count_sum += (double)counts[s] * b->coeffs[k];
                    ++k;
                }
            /* Q5: second loop, coeffIter never advances (peakcall.cpp:200) */
            for (uint16_t s = 0; s < b->n_expt; ++s)
                if (!b->control[s]) count_sum += (double)counts[s];
        }
    }
    if (count_sum != 0) {
        for (uint32_t j = 0; j < b->W; ++j) {
            cell *c = at(b, j);
            if (forward) c->f += b->kernel[j] * count_sum;
            else c->r += b->kernel[j] * count_sum;
        }
        cell *centre = at(b, b->bw);
        if (centre->hits) {
            for (uint16_t s = 0; s < b->n_expt; ++s) centre->hits[s] += counts[s];
        } else {
            centre->hits = (uint32_t *)xmalloc(b->n_expt * sizeof(uint32_t));
            memcpy(centre->hits, counts, b->n_expt * sizeof(uint32_t));
        }
    }
    b->buffer_pos = pos;
}

/* ProfileBuffer::flushContig, peakcall.cpp:224-231 */
uint64_t orc_buf_flush(orc_buf *b) {
    orc_buf_add(b, NULL, b->contig, (uint32_t)(b->buffer_pos + b->W), 1);
    b->buffer_pos = 0;
    b->last_pos = 0;
    const uint64_t res = b->n_contig_regions;
    b->n_contig_regions = 0;
    return res;
}

/* ---------------------------------------------------------------------- */
/* single-unit helpers for parity tests                                    */
/* ---------------------------------------------------------------------- */
typedef struct {
    orc_unit_region *out;
    uint32_t *sums;
    size_t cap, n;
    uint16_t n_expt;
} unit_sink;

static void fill_unit_region(unit_sink *u, orc_region *g, int accepted) {
    if (u->n < u->cap) {
        orc_unit_region *o = &u->out[u->n];
        o->left = g->left;
        o->npos = g->n;
        o->right = g->left + g->n - 1;
        o->peak = g->peak_pos;
        o->peak_score = g->peak_score;
        o->contig = g->contig;
        o->forward = g->forward;
        o->accepted = accepted;
        o->sum = orc_region_sum(g);
        o->kurtosis = g->n ? orc_region_kurtosis(g) : NAN;
        o->corr = orc_region_corr(g, 0);
        if (u->sums) orc_region_expt_sums(g, u->sums + u->n * u->n_expt);
    }
    u->n++;
}

static void unit_cb(void *user, orc_region *g) {
    fill_unit_region((unit_sink *)user, g, 1);
    orc_region_free(g);
}

static void unit_rej_cb(void *user, orc_region *g) {
    fill_unit_region((unit_sink *)user, g, 0);
    orc_region_free(g);
}

void orc_buf_set_reject_cb(orc_buf *b, orc_region_cb cb) { b->rej_cb = cb; }

int64_t orc_run_unit(const double *kernel, uint32_t kernel_size,
                     double region_thr, double kurt_thr, double corr_thr,
                     double hit_thr, int buffer_forward, int nondir,
                     uint16_t n_expt, const uint8_t *control,
                     const double *coeffs, uint32_t n_coeffs,
                     uint32_t contig, size_t n, const uint32_t *pos,
                     const uint32_t *counts_fwd, const uint32_t *counts_rev,
                     orc_unit_region *out, uint32_t *out_sums, size_t cap) {
    unit_sink u = {out, out_sums, cap, 0, n_expt};
    orc_buf *b = orc_buf_new(kernel, kernel_size, region_thr, kurt_thr,
                             corr_thr, hit_thr, buffer_forward, n_expt, control,
                             coeffs, n_coeffs, unit_cb, &u, NULL, NULL);
    b->rej_cb = unit_rej_cb;
    /* the unit belongs to `contig`; start the buffer there (no flush) */
    b->contig = contig;
    b->region->contig = contig;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t *cf = counts_fwd ? counts_fwd + i * n_expt : NULL;
        const uint32_t *cr = counts_rev ? counts_rev + i * n_expt : NULL;
        int any_f = 0, any_r = 0;
        for (uint16_t s = 0; s < n_expt; ++s) {
            if (cf && cf[s]) any_f = 1;
            if (cr && cr[s]) any_r = 1;
        }
        if (nondir) {
            if (any_f) orc_buf_add(b, cf, contig, pos[i], 1);
            if (any_r) orc_buf_add(b, cr, contig, pos[i], 0);
        } else {
            /* directional: one strand per buffer */
            const uint32_t *c = buffer_forward ? cf : cr;
            const int any = buffer_forward ? any_f : any_r;
            if (any) orc_buf_add(b, c, contig, pos[i], buffer_forward);
        }
    }
    orc_buf_flush(b);
    orc_buf_free(b);
    return (int64_t)u.n;
}

/* a synthetic unit generated and run inside the oracle (bench.py's genome
 * workloads at full size without host count matrices; see orc.h) */
int64_t orc_genome_unit(const double *kernel, uint32_t kernel_size, double region_thr,
                        double kurt_thr, double corr_thr, double hit_thr, int buffer_forward,
                        int nondir, uint16_t n_expt, const uint8_t *control,
                        const uint64_t *seeds, const uint8_t *with_peaks, uint64_t peak_seed,
                        const int32_t *offset, uint32_t contig, uint32_t len, uint16_t bw,
                        orc_unit_region *out, uint32_t *out_sums, size_t cap) {
    const int nstr = nondir ? 2 : 1;
    const size_t ntr = (size_t)nstr * n_expt;
    uint32_t **tp = (uint32_t **)xmalloc(ntr * sizeof(uint32_t *));
    uint32_t **tc = (uint32_t **)xmalloc(ntr * sizeof(uint32_t *));
    size_t *tn = (size_t *)xmalloc(ntr * sizeof(size_t));
    size_t *cur = (size_t *)calloc(ntr, sizeof(size_t));
    /* positions holding a tag of any track, as a bitmap over 1..len */
    uint64_t *bits = (uint64_t *)calloc((size_t)len / 64 + 2, sizeof(uint64_t));
    for (int k = 0; k < nstr; ++k) {
        const int strand = nondir ? k : (buffer_forward ? 0 : 1);
        for (uint16_t s = 0; s < n_expt; ++s) {
            const size_t t = (size_t)k * n_expt + s;
            const size_t need = orc_synth_track_ex(seeds[s], contig, strand, nondir, len, bw,
                                                   with_peaks[s], offset[strand], peak_seed, NULL,
                                                   NULL, 0);
            tp[t] = (uint32_t *)xmalloc((need + 1) * sizeof(uint32_t));
            tc[t] = (uint32_t *)xmalloc((need + 1) * sizeof(uint32_t));
            tn[t] = orc_synth_track_ex(seeds[s], contig, strand, nondir, len, bw, with_peaks[s],
                                       offset[strand], peak_seed, tp[t], tc[t], need);
            for (size_t i = 0; i < tn[t]; ++i) bits[tp[t][i] >> 6] |= 1ull << (tp[t][i] & 63);
        }
    }
    unit_sink u = {out, out_sums, cap, 0, n_expt};
    orc_buf *b = orc_buf_new(kernel, kernel_size, region_thr, kurt_thr, corr_thr, hit_thr,
                             buffer_forward, n_expt, control, NULL, 0, unit_cb, &u, NULL, NULL);
    b->rej_cb = unit_rej_cb;
    b->contig = contig;
    b->region->contig = contig;
    uint32_t *cv = (uint32_t *)xmalloc((size_t)nstr * n_expt * sizeof(uint32_t));
    for (size_t w = 0; w <= (size_t)len / 64 + 1; ++w) {
        uint64_t m = bits[w];
        while (m) {
            const uint32_t x = (uint32_t)(w * 64 + (size_t)__builtin_ctzll(m));
            m &= m - 1;
            for (int k = 0; k < nstr; ++k) {
                int any = 0;
                for (uint16_t s = 0; s < n_expt; ++s) {
                    const size_t t = (size_t)k * n_expt + s;
                    uint32_t c = 0;
                    if (cur[t] < tn[t] && tp[t][cur[t]] == x) c = tc[t][cur[t]++];
                    cv[(size_t)k * n_expt + s] = c;
                    any |= c != 0;
                }
                /* orc_run_unit's order: forward add, then reverse add */
                if (any)
                    orc_buf_add(b, cv + (size_t)k * n_expt, contig, x,
                                nondir ? k == 0 : buffer_forward);
            }
        }
    }
    orc_buf_flush(b);
    orc_buf_free(b);
    for (size_t t = 0; t < ntr; ++t) {
        free(tp[t]);
        free(tc[t]);
    }
    free(tp);
    free(tc);
    free(tn);
    free(cur);
    free(bits);
    free(cv);
    return (int64_t)u.n;
}

typedef struct {
    double *score;
    uint32_t len;
} prof_sink;

static void prof_cb(void *user, int forward, uint32_t contig, uint32_t pos,
                    double score) {
    (void)forward;
    (void)contig;
    prof_sink *p = (prof_sink *)user;
    if (pos >= 1 && pos <= p->len) p->score[pos - 1] = score;
}

int orc_unit_profile(const double *kernel, uint32_t kernel_size,
                     int buffer_forward, int nondir, uint16_t n_expt,
                     const uint8_t *control, const double *coeffs,
                     uint32_t n_coeffs, size_t n, const uint32_t *pos,
                     const uint32_t *counts_fwd, const uint32_t *counts_rev,
                     uint32_t len, double *score_out) {
    prof_sink p = {score_out, len};
    memset(score_out, 0, (size_t)len * sizeof(double));
    orc_buf *b = orc_buf_new(kernel, kernel_size, 1e300, 0, -1, 0,
                             buffer_forward, n_expt, control, coeffs, n_coeffs,
                             NULL, NULL, prof_cb, &p);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t *cf = counts_fwd ? counts_fwd + i * n_expt : NULL;
        const uint32_t *cr = counts_rev ? counts_rev + i * n_expt : NULL;
        int any_f = 0, any_r = 0;
        for (uint16_t s = 0; s < n_expt; ++s) {
            if (cf && cf[s]) any_f = 1;
            if (cr && cr[s]) any_r = 1;
        }
        if (nondir) {
            if (any_f) orc_buf_add(b, cf, 0, pos[i], 1);
            if (any_r) orc_buf_add(b, cr, 0, pos[i], 0);
        } else {
            const uint32_t *c = buffer_forward ? cf : cr;
            const int any = buffer_forward ? any_f : any_r;
            if (any) orc_buf_add(b, c, 0, pos[i], buffer_forward);
        }
    }
    orc_buf_flush(b);
    orc_buf_free(b);
    return 0;
}
