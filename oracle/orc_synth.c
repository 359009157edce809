/*
 * oracle/orc_synth.c -- TEST INFRASTRUCTURE ONLY (see orc.h header).
 *
 * Host side of the synthetic hg19-shaped input spec (DESIGN.md "Synthetic
 * input", after SURVEY.md 8(d)): per-position Poisson background from a
 * counter-based hash, plus peaks whose tag offsets are an integer
 * Irwin-Hall approximation of N(0, 60).  Everything is integer arithmetic
 * so the device generator reproduces it exactly.  Also the timed CPU
 * baseline driver for bench.py.
 */
#include "orc.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define SYN_LAMBDA 0.002925

void orc_synth_thresholds(double lambda, uint64_t *t) {
    double p = exp(-lambda), cdf = p;
    for (int k = 0; k < 6; ++k) {
        t[k] = cdf >= 1.0 ? ~0ull : (uint64_t)(cdf * 18446744073709551616.0);
        p *= lambda / (double)(k + 1);
        cdf += p;
    }
}

typedef struct {
    uint32_t pos;
} ptag;

static int cmp_u32(const void *a, const void *b) {
    const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

size_t orc_synth_track(uint64_t seed, uint32_t contig, int strand, int nondir,
                       uint32_t len, uint16_t bw, int with_peaks,
                       uint32_t *pos, uint32_t *cnt, size_t cap) {
    return orc_synth_track_ex(seed, contig, strand, nondir, len, bw, with_peaks, 0, 0, pos, cnt,
                              cap);
}

/* offset: the track moved as the wiggle reader's -s moves it (forward +s,
 * reverse -s, misc/format.cpp:693-705), counts leaving [1, len] dropped.
 * peak_seed != 0: replicate samples -- centres from peak_seed's keys, shared
 * by every sample; per-sample height and a -20..+20 centre jitter from the
 * sample's own seed (device: up_unit_synth_ex). */
size_t orc_synth_track_ex(uint64_t seed, uint32_t contig, int strand, int nondir,
                          uint32_t len, uint16_t bw, int with_peaks, int32_t offset,
                          uint64_t peak_seed, uint32_t *pos, uint32_t *cnt, size_t cap) {
    const uint64_t skey = mix64(seed);
    const uint64_t ckey = mix64(skey ^ (uint64_t)(contig + 1));
    const uint64_t tkey = mix64(ckey ^ (uint64_t)(0x100 + strand));
    const uint64_t pckey = peak_seed ? mix64(mix64(peak_seed) ^ (uint64_t)(contig + 1)) : ckey;
    const uint64_t pkey = mix64(pckey ^ (uint64_t)(0x200 + (nondir ? 0 : strand)));
    const int64_t lo = 2 * (int64_t)bw + 2, hi = (int64_t)len - 2 * (int64_t)bw - 1;
    uint64_t thr[6];
    orc_synth_thresholds(SYN_LAMBDA, thr);

    /* peak tags */
    uint32_t *tags = NULL;
    size_t ntags = 0, tcap = 0;
    if (with_peaks && hi >= lo) {
        uint32_t npk = len / 150000u;
        if (npk < 1) npk = 1;
        int64_t clo, chi;
        if (len >= 20000u + 1u) { clo = 10000; chi = (int64_t)len - 10000; }
        else { clo = 2 * (int64_t)bw + 200; chi = (int64_t)len - 2 * (int64_t)bw - 200; }
        const int64_t shift = (nondir && strand == 1) ? 150 : 0;
        for (uint32_t j = 0; chi >= clo && j < npk; ++j) {
            const uint64_t h = mix64(pkey ^ mix64(0x7065616B00000000ull + j));
            int64_t centre = clo + (int64_t)(h % (uint64_t)(chi - clo + 1));
            uint32_t n = 20u + (uint32_t)(mix64(h) % 180u);
            // replicate mode: the shared hash also picks the peak's kind --
            // 0/1 an artifact on strand 0/1 only, 2 a spike (every tag of every
            // sample at the shared centre), 3 a weak peak (2..11 tags per sample), else normal
            const uint32_t kind = peak_seed ? (uint32_t)(h >> 56) & 15u : 4u;
            if (peak_seed) {
                const uint64_t hs = mix64(h ^ skey);
                n = 20u + (uint32_t)(hs % 180u);
                if (kind != 2) centre += (int64_t)((hs >> 32) % 41u) - 20;
                if (kind == 3) n = 2u + (uint32_t)(hs % 10u);
                if (kind <= 1 && (uint32_t)strand != kind) n = 0;
            }
            for (uint32_t i = 0; i < n; ++i) {
                int64_t s = 0;
                const uint64_t base = mix64(tkey ^ h ^ mix64(0x74616700000000ull + i));
                for (int m = 0; m < 12; ++m) s += (int64_t)(mix64(base + (uint64_t)m) >> 32);
                const int64_t num = 60 * (s - 6 * 4294967296ll);
                const int64_t off = kind == 2 ? 0 : (num + 2147483648ll) >> 32; /* floor */
                const int64_t p = centre + shift + off;
                if (p < lo || p > hi || p + offset < 1 || p + offset > (int64_t)len) continue;
                if (ntags == tcap) {
                    tcap = tcap ? 2 * tcap : 1024;
                    tags = (uint32_t *)realloc(tags, tcap * sizeof(uint32_t));
                }
                tags[ntags++] = (uint32_t)p;
            }
        }
    }
    size_t out = 0, ti = 0;
    if (peak_seed) {
        /* replicate mode's background: chunks of 2^16 positions, each with
         * n ~ Poisson(lambda * 2^16) tags at uniform positions (n = #{k :
         * tab[k] <= u0}); device: synth_bgc_kernel */
        uint64_t tab[1024];
        const double mu = SYN_LAMBDA * 65536.0;
        double pr = exp(-mu), cdf = pr;
        for (int k = 0; k < 1024; ++k) {
            tab[k] = cdf >= 1.0 ? ~0ull : (uint64_t)(cdf * 18446744073709551616.0);
            pr *= mu / (double)(k + 1);
            cdf += pr;
        }
        const uint64_t nch = hi >= lo ? ((uint64_t)(hi - lo + 1) + 65535) >> 16 : 0;
        for (uint64_t ch = 0; ch < nch; ++ch) {
            const uint64_t u0 = mix64(tkey ^ mix64(0x6267000000000000ull + ch));
            uint32_t a = 0, b = 1024;
            while (a < b) {
                const uint32_t m = (a + b) >> 1;
                if (tab[m] <= u0) a = m + 1;
                else b = m;
            }
            const int64_t base = lo + (int64_t)(ch << 16);
            for (uint32_t i = 0; i < a; ++i) {
                const int64_t x = base + (int64_t)(mix64(u0 ^ mix64((uint64_t)i + 1)) >> 48);
                if (x > hi || x + offset < 1 || x + offset > (int64_t)len) continue;
                if (ntags == tcap) {
                    tcap = tcap ? 2 * tcap : 1024;
                    tags = (uint32_t *)realloc(tags, tcap * sizeof(uint32_t));
                }
                tags[ntags++] = (uint32_t)x;
            }
        }
        qsort(tags, ntags, sizeof(uint32_t), cmp_u32);
        while (ti < ntags) {
            const uint32_t x = tags[ti];
            uint32_t c = 0;
            while (ti < ntags && tags[ti] == x) { ++c; ++ti; }
            if (out < cap) { pos[out] = (uint32_t)((int64_t)x + offset); cnt[out] = c; }
            ++out;
        }
        free(tags);
        return out;
    }
    if (ntags) qsort(tags, ntags, sizeof(uint32_t), cmp_u32);
    for (int64_t x = lo; x <= hi; ++x) {
        const uint64_t u = mix64(tkey ^ mix64((uint64_t)x));
        uint32_t c = 0;
        while (c < 6 && u >= thr[c]) ++c;
        while (ti < ntags && tags[ti] == (uint32_t)x) { ++c; ++ti; }
        if (c && x + offset >= 1 && x + offset <= (int64_t)len) {
            if (out < cap) { pos[out] = (uint32_t)(x + offset); cnt[out] = c; }
            ++out;
        }
    }
    free(tags);
    return out;
}

int orc_baseline_run(uint32_t n_contigs, const uint32_t *lens, uint64_t seed,
                     uint16_t bw, double region_thr, double kurt_thr,
                     double hit_thr, double background, uint64_t *n_pass,
                     uint64_t *n_reject, double *seconds) {
    const uint32_t W = 2u * bw + 1;
    double *k = (double *)malloc(W * sizeof(double));
    orc_kernel(bw, 1 / background, k);
    uint8_t ctl = 0;
    orc_buf *b[2];
    for (int s = 0; s < 2; ++s)
        b[s] = orc_buf_new(k, W, region_thr, kurt_thr, -1, hit_thr, s == 0, 1, &ctl,
                           NULL, 0, NULL, NULL, NULL, NULL);
    double t = 0;
    for (int s = 0; s < 2; ++s) {
        for (uint32_t c = 0; c < n_contigs; ++c) {
            const size_t cap = (size_t)(lens[c] / 64) + 4096;
            uint32_t *pos = (uint32_t *)malloc(cap * sizeof(uint32_t));
            uint32_t *cnt = (uint32_t *)malloc(cap * sizeof(uint32_t));
            size_t n = orc_synth_track(seed, c, s, 0, lens[c], bw, 1, pos, cnt, cap);
            if (n > cap) n = cap;
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            for (size_t i = 0; i < n; ++i) orc_buf_add(b[s], &cnt[i], c, pos[i], s == 0);
            orc_buf_flush(b[s]);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            t += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
            free(pos);
            free(cnt);
        }
    }
    *n_pass = orc_buf_nregions(b[0]) + orc_buf_nregions(b[1]);
    *n_reject = orc_buf_nrejects(b[0]) + orc_buf_nrejects(b[1]);
    *seconds = t;
    orc_buf_free(b[0]);
    orc_buf_free(b[1]);
    free(k);
    return 0;
}

/* One (contig, strand) unit of the hot-path baseline on its own buffer
 * (flushContig resets the position state, misc/peakcall.cpp:224-231, so
 * units are independent -- the reference's contig-subset method, README:37,
 * run as threads) over pre-generated hits: only the add/flush calls run. */
int orc_baseline_unit(const uint32_t *pos, const uint32_t *cnt, size_t n, uint32_t contig,
                      int strand, uint16_t bw, double region_thr, double kurt_thr,
                      double hit_thr, double background, uint64_t *n_pass,
                      uint64_t *n_reject) {
    const uint32_t W = 2u * bw + 1;
    double *k = (double *)malloc(W * sizeof(double));
    orc_kernel(bw, 1 / background, k);
    uint8_t ctl = 0;
    orc_buf *b = orc_buf_new(k, W, region_thr, kurt_thr, -1, hit_thr, strand == 0, 1, &ctl,
                             NULL, 0, NULL, NULL, NULL, NULL);
    for (size_t i = 0; i < n; ++i) orc_buf_add(b, &cnt[i], contig, pos[i], strand == 0);
    orc_buf_flush(b);
    *n_pass = orc_buf_nregions(b);
    *n_reject = orc_buf_nrejects(b);
    orc_buf_free(b);
    free(k);
    return 0;
}

/* Wiggle data lines "pos count\n" (or "pos -count\n" for a reverse track,
 * misc/format.cpp:1164-1219) for the test fixtures' synthetic wig files.
 * out must hold 24 bytes per pair; returns the bytes written. */
size_t orc_format_pairs(const uint32_t *pos, const uint32_t *cnt, size_t n, int neg,
                        char *out) {
    char *o = out;
    for (size_t i = 0; i < n; ++i) {
        char t[12];
        int m = 0;
        uint32_t v = pos[i];
        do { t[m++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (m) *o++ = t[--m];
        *o++ = ' ';
        if (neg) *o++ = '-';
        v = cnt[i];
        do { t[m++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (m) *o++ = t[--m];
        *o++ = '\n';
    }
    return (size_t)(o - out);
}
