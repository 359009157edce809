/*
 * oracle/orc_io.c -- TEST INFRASTRUCTURE ONLY (see orc.h header).
 *
 * Plain-C restatement of the reference's boundary layer for the hot path:
 * contig table (misc/format.cpp:27-57, misc/data.cpp:196-261), the wiggle
 * line parser and its stream wrappers (misc/format.cpp:242-683, 693-705,
 * 737-766, 798-811, 814-935), and the three CLI drivers (src/regions.cpp,
 * src/strand_shift.cpp, src/tags_in_regions.cpp), including the output
 * formats (misc/format.cpp:1141-1162, misc/filterstream.cpp:134-137).
 * Only wiggle input is restated (alignment formats feed convert_align,
 * which is outside the scope of the path).
 *
 * Deliberate choice (quirk Q18): NondirParseAlignStream's own
 * Alignment has an uninitialised `forward` member (format.cpp:819-825 never
 * sets it), so the reference's first merge step is undefined behaviour.  We
 * restate the intended two-handle merge (as if `forward` started true).
 */
#define _GNU_SOURCE 1 /* fopencookie */
#include "orc.h"

#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* ---------------------------------------------------------------------- */
/* small utilities                                                         */
/* ---------------------------------------------------------------------- */
static void fail(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    exit(1);
}

static void *xcalloc(size_t n, size_t sz) {
    void *p = calloc(n ? n : 1, sz ? sz : 1);
    if (!p) fail("oracle: out of memory\n");
    return p;
}

static char *xstrdup(const char *s) {
    char *p = strdup(s);
    if (!p) fail("oracle: out of memory\n");
    return p;
}

typedef struct {
    char *p;
    size_t n, cap;
} sbuf; /* growable output string */

static void sb_add(sbuf *b, const char *s, size_t n) {
    if (b->n + n + 1 > b->cap) {
        size_t c = b->cap ? b->cap : 256;
        while (c < b->n + n + 1) c *= 2;
        b->p = (char *)realloc(b->p, c);
        if (!b->p) fail("oracle: out of memory\n");
        b->cap = c;
    }
    memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void sb_puts(sbuf *b, const char *s) { sb_add(b, s, strlen(s)); }
static void sb_printf(sbuf *b, const char *fmt, ...) {
    char tmp[512];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    sb_add(b, tmp, (size_t)n);
}
/* OutStream << double: boost::lexical_cast, 17 significant digits
 * (misc/filterstream.cpp:134-137) */
static void sb_lex(sbuf *b, double v) { sb_printf(b, "%.17g", v); }
/* std::ostream << double with default precision 6 */
static void sb_os(sbuf *b, double v) { sb_printf(b, "%g", v); }

/* boost::lexical_cast<unsigned integer>: optional sign, digits only,
 * '-' wraps (two's complement).  Returns 0 on failure. */
static int lex_u64(const char *s, size_t n, uint64_t maxv, uint64_t *out) {
    size_t i = 0;
    int neg = 0;
    if (n == 0) return 0;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i == n) return 0;
    uint64_t v = 0;
    for (; i < n; ++i) {
        if (s[i] < '0' || s[i] > '9') return 0;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (maxv - d) / 10) return 0;
        v = v * 10 + d;
    }
    if (neg) v = (uint64_t)(-(int64_t)v) & maxv;
    *out = v;
    return 1;
}

static int lex_short(const char *s, short *out) {
    char *e;
    errno = 0;
    long v = strtol(s, &e, 10);
    if (*s == 0 || *e || errno || v < -32768 || v > 32767 || isspace((unsigned char)*s)) return 0;
    *out = (short)v;
    return 1;
}

static int lex_double(const char *s, double *out) {
    char *e;
    if (*s == 0 || isspace((unsigned char)*s)) return 0;
    double v = strtod(s, &e);
    if (*e) return 0;
    *out = v;
    return 1;
}

/* boost::tokenizer<char_separator<char>>(",") -- empty tokens dropped */
static int split_csv(const char *s, char ***out) {
    int n = 0, cap = 8;
    char **v = (char **)xcalloc((size_t)cap, sizeof(char *));
    const char *p = s;
    while (*p) {
        const char *q = strchr(p, ',');
        size_t len = q ? (size_t)(q - p) : strlen(p);
        if (len) {
            if (n == cap) { cap *= 2; v = (char **)realloc(v, (size_t)cap * sizeof(char *)); }
            v[n] = (char *)xcalloc(len + 1, 1);
            memcpy(v[n], p, len);
            ++n;
        }
        if (!q) break;
        p = q + 1;
    }
    *out = v;
    return n;
}

/* getFnamePrefix, misc/format.cpp:60-67 */
static char *fname_prefix(const char *name) {
    const char *slash = strrchr(name, '/');
    const char *b = slash ? slash + 1 : name;
    char *r = xstrdup(b);
    char *dot = strchr(r, '.');
    if (dot) *dot = 0;
    return r;
}

/* ---------------------------------------------------------------------- */
/* contig table: misc/format.cpp:27-57, misc/data.cpp:204-253              */
/* ---------------------------------------------------------------------- */
typedef struct {
    uint32_t n;
    char **names;
    uint32_t *sizes;
    uint32_t genome; /* uint32: wraps for hg19+mm9 (Q10) */
} ctab;

static int is_word(int c) { return isalnum(c) || c == '_'; }

static uint32_t ctab_find(const ctab *t, const char *name, size_t len) {
    for (uint32_t i = 0; i < t->n; ++i)
        if (strlen(t->names[i]) == len && memcmp(t->names[i], name, len) == 0) return i;
    return t->n;
}

/* misc/filterstream.cpp:30-50, 86-104: a name ending in GZIP_SUFFIX ".gz"
 * (misc/defaults.hpp:26) is read / written through boost's gzip filters --
 * here zlib behind a stdio cookie; BZIP2_SUFFIX ".bz2" takes bzip2 filters,
 * refused in this image (no libbz2 headers) with an error exit. */
static int ends_with(const char *s, const char *suf) {
    const size_t n = strlen(s), m = strlen(suf);
    return n >= m && strcmp(s + n - m, suf) == 0;
}
static ssize_t gzc_read(void *c, char *buf, size_t n) {
    const int r = gzread((gzFile)c, buf, (unsigned)(n < (1u << 30) ? n : (1u << 30)));
    if (r < 0) fail("error: gzip stream error\n\n");
    return r;
}
static ssize_t gzc_write(void *c, const char *buf, size_t n) {
    size_t done = 0;
    while (done < n) {
        const size_t k = n - done < (1u << 30) ? n - done : (1u << 30);
        const int w = gzwrite((gzFile)c, buf + done, (unsigned)k);
        if (w <= 0) return done ? (ssize_t)done : -1;
        done += (size_t)w;
    }
    return (ssize_t)done;
}
static int gzc_close(void *c) { return gzclose((gzFile)c) == Z_OK ? 0 : EOF; }
static FILE *filter_open(const char *fname, int write) {
    if (ends_with(fname, ".bz2"))
        fail("error: could not %s %s: bzip2 (.bz2) streams are not supported by this build "
             "(libbz2 headers absent)\n", write ? "write" : "read", fname);
    if (!ends_with(fname, ".gz")) return fopen(fname, write ? "wb" : "rb");
    gzFile g = gzopen(fname, write ? "wb" : "rb");
    if (!g) return NULL;
    if (!write) {  /* boost's gzip_decompressor throws on a file without a gzip header */
        char c;
        const int r = gzread(g, &c, 1);
        if (r == 1 && gzdirect(g)) fail("error: could not read %s: not in gzip format\n\n", fname);
        if (r == 1) gzungetc((unsigned char)c, g);
    }
    cookie_io_functions_t io = {write ? NULL : gzc_read, write ? gzc_write : NULL, NULL, gzc_close};
    FILE *f = fopencookie(g, write ? "w" : "r", io);
    if (!f) gzclose(g);
    return f;
}

/* line reader with std::getline/istream::good() semantics */
typedef struct {
    FILE *fp;
    char *fname;
    uint64_t line_no;
    int eof, open;
    char *buf;
    size_t cap;
} instream;

static void in_open(instream *s, const char *fname) {
    memset(s, 0, sizeof *s);
    if (strcmp(fname, "stdin") == 0) {
        s->fp = stdin;
        s->fname = xstrdup("standard input stream");
    } else {
        s->fp = filter_open(fname, 0);
        if (!s->fp) fail("error: could not read %s\n\n", fname);
        s->fname = xstrdup(fname);
    }
    s->open = 1;
}
static int in_good(const instream *s) { return s->open && !s->eof; }
static void in_close(instream *s) {
    if (s->open && s->fp && s->fp != stdin) fclose(s->fp);
    s->open = 0;
}
/* returns the line (without '\n'); "" and eof once exhausted */
static const char *in_read_line(instream *s, size_t *len) {
    ssize_t n = getline(&s->buf, &s->cap, s->fp);
    s->line_no++;
    if (n < 0) {
        s->eof = 1;
        if (!s->buf) { s->cap = 1; s->buf = (char *)xcalloc(1, 1); }
        s->buf[0] = 0;
        *len = 0;
        return s->buf;
    }
    if (n > 0 && s->buf[n - 1] == '\n') s->buf[--n] = 0;
    else s->eof = 1; /* last line without newline sets eofbit */
    *len = (size_t)n;
    return s->buf;
}

static ctab *ctab_parse(const char *fname) {
    fprintf(stderr, "reading %s... ", fname);
    ctab *t = (ctab *)xcalloc(1, sizeof *t);
    uint32_t cap = 64;
    t->names = (char **)xcalloc(cap, sizeof(char *));
    t->sizes = (uint32_t *)xcalloc(cap, sizeof(uint32_t));
    instream in;
    in_open(&in, fname);
    while (in_good(&in)) {
        size_t len;
        const char *l = in_read_line(&in, &len);
        if (!len || l[0] == '#') continue;
        /* regex ^(\w+)\W+(\d+) */
        size_t i = 0;
        while (i < len && is_word((unsigned char)l[i])) ++i;
        if (i == 0) continue;
        size_t j = i;
        while (j < len && !is_word((unsigned char)l[j])) ++j;
        if (j == i) continue;
        size_t k = j;
        while (k < len && isdigit((unsigned char)l[k])) ++k;
        if (k == j) continue;
        uint64_t size;
        if (!lex_u64(l + j, k - j, 0xFFFFFFFFull, &size)) {
            fprintf(stderr, "terminate called after throwing bad_lexical_cast\n");
            abort();
        }
        if (ctab_find(t, l, i) != t->n) {
            char *nm = (char *)xcalloc(i + 1, 1);
            memcpy(nm, l, i);
            fail("error: %s defined twice in contig table\n\n", nm);
        }
        if (t->n == cap) {
            cap *= 2;
            t->names = (char **)realloc(t->names, cap * sizeof(char *));
            t->sizes = (uint32_t *)realloc(t->sizes, cap * sizeof(uint32_t));
        }
        t->names[t->n] = (char *)xcalloc(i + 1, 1);
        memcpy(t->names[t->n], l, i);
        t->sizes[t->n] = (uint32_t)size;
        t->genome += (uint32_t)size;
        t->n++;
    }
    in_close(&in);
    if (t->n == 0) fail("error: no contigs in table\n\n");
    fprintf(stderr, "%u contigs\n", t->n);
    return t;
}

/* ---------------------------------------------------------------------- */
/* wiggle parser: misc/format.cpp:242-272, 503-565, 654-705, 737-766        */
/* ---------------------------------------------------------------------- */
enum { FMT_NONE = 0, FMT_DIRWIG = 6, FMT_NONDIRWIG = 7 };

typedef struct {
    int forward;
    uint32_t contig, first, last, count;
} align_t;

typedef struct pstream {
    instream in;
    char *fname_arg;
    const ctab *ct;
    int format;
    align_t a;
    char *name;
    uint64_t total, oob, confident, expected;
    short offset;
    uint16_t use_len;
    /* 0: plain ParseAlignStream, 1/2: StrandParseAlignStream fwd/rev */
    int strand_mode;
} pstream;

static void ps_error(const pstream *p, const char *msg) {
    fail("error: %s in %s line %llu\n\n", msg, p->in.fname,
         (unsigned long long)p->in.line_no);
}

static void ps_open(pstream *p, const char *fname, const ctab *ct, short offset,
                    uint16_t use_len, int strand_mode) {
    memset(p, 0, sizeof *p);
    in_open(&p->in, fname);
    p->fname_arg = xstrdup(fname);
    p->ct = ct;
    p->offset = offset;
    p->use_len = use_len;
    p->strand_mode = strand_mode;
    p->name = fname_prefix(fname);
    p->a.forward = 1;
    p->a.contig = ct->n; /* ctor: Alignment(true, size, 0, 0, "", 0); open() sets 0 */
    p->a.contig = 0;
}

/* NAME_REGEX1 name="(.+?)" (format.hpp:32): first occurrence of name=" with
 * at least one character before a closing quote; returns malloc'd or NULL */
static char *name_regex1(const char *l) {
    for (const char *p = strstr(l, "name=\""); p; p = strstr(p + 1, "name=\"")) {
        const char *q = p + 6;
        if (!*q) continue;
        const char *e = strchr(q + 1, '"');
        if (!e) continue;
        char *r = (char *)xcalloc((size_t)(e - q) + 1, 1);
        memcpy(r, q, (size_t)(e - q));
        return r;
    }
    return NULL;
}

/* NAME_REGEX2 name=(.+?)<space> (format.hpp:33) */
static char *name_regex2(const char *l) {
    for (const char *p = strstr(l, "name="); p; p = strstr(p + 1, "name=")) {
        const char *q = p + 5;
        if (!*q) continue;
        const char *e = strchr(q + 1, ' ');
        if (!e) continue;
        char *r = (char *)xcalloc((size_t)(e - q) + 1, 1);
        memcpy(r, q, (size_t)(e - q));
        return r;
    }
    return NULL;
}

static char *track_name(const char *l, int *ok) {
    char *r = name_regex1(l);
    if (!r) r = name_regex2(l);
    *ok = r != NULL;
    return r ? r : xstrdup("");
}

/* DIRECTIONAL_WIG_NAME_REGEX "(.+) ([+-])": greedy -> last " +"/" -" with a
 * non-empty prefix.  Returns 1 and splits when it matches. */
static int dir_name(const char *name, char **expt, int *fwd) {
    size_t n = strlen(name);
    for (size_t i = n >= 2 ? n - 2 : 0; n >= 2; --i) {
        if (i >= 1 && name[i] == ' ' && (name[i + 1] == '+' || name[i + 1] == '-')) {
            *expt = (char *)xcalloc(i + 1, 1);
            memcpy(*expt, name, i);
            *fwd = name[i + 1] == '+';
            return 1;
        }
        if (i == 0) break;
    }
    return 0;
}

static int starts_with(const char *l, const char *p) { return strncmp(l, p, strlen(p)) == 0; }

static void ps_parse(pstream *p, const char *l, size_t len) {
    char *nm1 = NULL;
    p->a.count = 0;
    if (len == 0 || l[0] == '#') return;
    if (p->format == FMT_NONE) {
        if (starts_with(l, "track")) {
            int ok;
            char *nm = track_name(l, &ok);
            if (ok) { free(p->name); p->name = xstrdup(nm); }
            if (strstr(l, "type=wiggle_0")) {
                char *e;
                int fwd;
                if (dir_name(p->name, &e, &fwd)) {
                    p->format = FMT_DIRWIG;
                    free(p->name);
                    p->name = e;
                    p->a.forward = fwd;
                } else {
                    p->format = FMT_NONDIRWIG;
                    free(p->name);
                    p->name = xstrdup(nm);
                    p->a.forward = 1;
                }
            } else {
                fail("oracle: non-wiggle input (%s) is outside the restated path\n", p->in.fname);
            }
            free(nm);
            return;
        }
        fail("oracle: non-wiggle input (%s) is outside the restated path\n", p->in.fname);
    }
    if (isdigit((unsigned char)l[0])) {
        if (p->a.contig == p->ct->n) return;
        size_t d = len;
        while (d > 0 && l[d - 1] != '\t' && l[d - 1] != ' ') --d;
        if (d == 0) ps_error(p, "bad format");
        --d; /* delimiter index */
        uint64_t pos, cnt;
        if (!lex_u64(l, d, 0xFFFFFFFFull, &pos)) ps_error(p, "bad format");
        size_t cs = d + (l[d + 1] == '-' ? 2 : 1);
        if (!lex_u64(l + cs, len - cs, 0xFFFFFFFFull, &cnt)) ps_error(p, "bad format");
        p->a.first = (uint32_t)pos;
        p->a.count = (uint32_t)cnt;
        if (p->format == FMT_DIRWIG)
            p->a.last = p->a.first + (p->use_len == 0 ? 0u
                        : (p->a.forward ? (uint32_t)(p->use_len - 1) : (uint32_t)-(int32_t)(p->use_len - 1)));
        else
            p->a.last = p->a.first + (p->use_len == 0 ? 0u : (uint32_t)(p->use_len - 1));
        p->total += p->a.count;
    } else if (starts_with(l, "variableStep chrom=") && len > 19) {
        p->a.contig = ctab_find(p->ct, l + 19, len - 19);
        return;
    } else if (starts_with(l, "track") && (nm1 = name_regex1(l)) != NULL) {
        char *nm = nm1;
        p->a.contig = p->ct->n;
        free(p->name);
        p->name = nm;
        if (p->format == FMT_DIRWIG) {
            char *e;
            int fwd;
            if (!dir_name(p->name, &e, &fwd)) ps_error(p, "strand not defined");
            free(p->name);
            p->name = e;
            p->a.forward = fwd;
        }
        return;
    } else {
        ps_error(p, "bad format");
    }
    /* offset and bounds, format.cpp:654-678 */
    if (p->a.count != 0 && p->a.contig != p->ct->n) {
        const uint16_t read_len = p->use_len;
        if (read_len != 0)
            p->a.last = p->a.first + (p->a.forward ? (uint32_t)(read_len - 1) : (uint32_t)-(int32_t)(read_len - 1));
        if (p->offset != 0) {
            if ((p->a.forward && ((int)p->a.first > -p->offset)) ||
                ((!p->a.forward) && ((int)p->a.last > p->offset))) {
                p->a.first += (uint32_t)(p->a.forward ? p->offset : -p->offset);
                p->a.last += (uint32_t)(p->a.forward ? p->offset : -p->offset);
            } else {
                p->oob += p->a.count;
                p->a.count = 0;
                return;
            }
        }
        const uint32_t size = p->ct->sizes[p->a.contig];
        if (p->a.first == 0 || p->a.first > size || p->a.last == 0 || p->a.last > size) {
            p->oob += p->a.count;
            p->a.count = 0;
            return;
        }
        p->confident += p->a.count;
    }
}

/* ParseAlignStream::readAlign, format.cpp:693-705 */
static void ps_read_align_plain(pstream *p) {
    size_t len;
    if (in_good(&p->in)) {
        const char *l = in_read_line(&p->in, &len);
        ps_parse(p, l, len);
    } else {
        p->a.count = 0;
        p->a.contig = p->ct->n;
    }
    while ((p->a.count == 0 || p->a.contig == p->ct->n) && in_good(&p->in)) {
        const char *l = in_read_line(&p->in, &len);
        ps_parse(p, l, len);
    }
}

/* StrandParseAlignStream::readAlign, format.cpp:798-811 */
static void ps_read_align(pstream *p) {
    ps_read_align_plain(p);
    if (p->strand_mode == 0) return;
    const int want_fwd = p->strand_mode == 1;
    if (p->format == FMT_DIRWIG && want_fwd && !p->a.forward && p->a.count > 0) {
        p->a.count = 0;
        in_close(&p->in);
    }
    while (in_good(&p->in) && p->a.forward != want_fwd) ps_read_align_plain(p);
}

/* ParseAlignStream::getExpectedTags, format.cpp:737-766 */
static uint64_t ps_expected(pstream *p) {
    if (p->expected == 0) {
        while (in_good(&p->in)) {
            size_t len;
            const char *l = in_read_line(&p->in, &len);
            if (len && l[0] == '#') {
                const char *m = strstr(l, "# tags=");
                if (m && isdigit((unsigned char)m[7])) {
                    size_t k = 7;
                    while (isdigit((unsigned char)m[k])) ++k;
                    uint64_t v;
                    if (!lex_u64(m + 7, k - 7, ~0ull, &v)) abort();
                    if (p->expected == 0) p->expected = v;
                    else ps_error(p, "multiple tag count headers");
                    if (p->expected == 0) ps_error(p, "zero tag count");
                }
            } else {
                char *copy = (char *)xcalloc(len + 1, 1);
                memcpy(copy, l, len);
                ps_parse(p, copy, len);
                free(copy);
                if (p->expected == 0) {
                    pstream t;
                    ps_open(&t, p->fname_arg, p->ct, p->offset, p->use_len, 0);
                    while (in_good(&t.in)) ps_read_align_plain(&t);
                    p->expected = t.confident;
                    in_close(&t.in);
                }
                break;
            }
        }
    }
    return p->expected;
}

/* ---------------------------------------------------------------------- */
/* polymorphic stream: ParseAlignStream or NondirParseAlignStream           */
/* ---------------------------------------------------------------------- */
typedef struct {
    int nondir;
    pstream p;        /* directional */
    pstream f, r;     /* nondirectional halves */
    align_t a;        /* merged head (nondir) */
    uint64_t expected;
} stream_t;

static void st_open(stream_t *s, const char *fname, const ctab *ct, short offset,
                    uint16_t use_len, int nondir) {
    memset(s, 0, sizeof *s);
    s->nondir = nondir;
    if (!nondir) {
        ps_open(&s->p, fname, ct, offset, use_len, 0);
    } else {
        ps_open(&s->f, fname, ct, offset, use_len, 1);
        ps_open(&s->r, fname, ct, offset, use_len, 2);
        s->a.forward = 1; /* Q18: intended merge */
        s->a.contig = ct->n;
    }
}

static pstream *st_further(stream_t *s) {
    return s->f.in.line_no >= s->r.in.line_no ? &s->f : &s->r;
}

static uint64_t st_expected(stream_t *s) {
    if (!s->nondir) return ps_expected(&s->p);
    if (s->expected == 0) s->expected = ps_expected(st_further(s));
    return s->expected;
}

static int which_lower(const stream_t *s) {
    const align_t *a1 = &s->f.a, *a2 = &s->r.a;
    switch (2 * (a1->count == 0) + (a2->count == 0)) {
    case 0:
        if (a1->contig == a2->contig) return a1->first <= a2->first;
        return a1->contig < a2->contig;
    case 1: return 1;
    case 2: return 0;
    default: return 1;
    }
}

/* NondirParseAlignStream::readAlign, format.cpp:873-895 */
static const align_t *st_read(stream_t *s) {
    if (!s->nondir) {
        ps_read_align(&s->p);
        return &s->p.a;
    }
    if (s->a.forward) {
        ps_read_align(&s->f);
        if (s->f.a.forward && s->f.a.contig == s->a.contig && s->f.a.first < s->a.first) {
            fprintf(stderr, "%u\t%u\n", s->f.a.first, s->a.first);
            ps_error(&s->f, "alignments out of order");
        }
    } else {
        ps_read_align(&s->r);
        if (!s->r.a.forward && s->r.a.contig == s->a.contig && s->r.a.first < s->a.first)
            ps_error(&s->r, "alignments out of order");
    }
    if (s->f.in.line_no == 0) ps_read_align(&s->f);
    if (s->r.in.line_no == 0) ps_read_align(&s->r);
    s->a = which_lower(s) ? s->f.a : s->r.a;
    return &s->a;
}

static const align_t *st_last(const stream_t *s) { return s->nondir ? &s->a : &s->p.a; }
static const char *st_name(stream_t *s) { return s->nondir ? st_further(s)->name : s->p.name; }
static uint64_t st_confident(stream_t *s) { return s->nondir ? st_further(s)->confident : s->p.confident; }
static uint64_t st_oob(stream_t *s) { return s->nondir ? st_further(s)->oob : s->p.oob; }

/* ---------------------------------------------------------------------- */
/* TCLAP-like argument handling (only the "-x value" / "--long value" forms) */
/* ---------------------------------------------------------------------- */
typedef struct {
    const char *sflag, *lflag;
    int is_switch, required, seen;
    const char *value;
} argspec;

static int parse_args(int argc, char **argv, argspec *specs, int nspec,
                      char ***pos, int *npos) {
    *pos = (char **)xcalloc((size_t)argc + 1, sizeof(char *));
    *npos = 0;
    int only_pos = 0;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        if (!only_pos && strcmp(a, "--") == 0) { only_pos = 1; continue; }
        if (!only_pos && (strcmp(a, "--version") == 0 || strcmp(a, "-v") == 0)) {
            printf("\n%s  version: 1.0\n\n", argv[0]);
            exit(0);
        }
        if (!only_pos && (strcmp(a, "--help") == 0 || strcmp(a, "-h") == 0)) {
            printf("See README.TXT for more information\n");
            exit(0);
        }
        if (!only_pos && a[0] == '-' && a[1] != 0) {
            int matched = 0;
            for (int k = 0; k < nspec && !matched; ++k) {
                argspec *s = &specs[k];
                int hit = (a[1] != '-' && s->sflag && strcmp(a + 1, s->sflag) == 0) ||
                          (a[1] == '-' && s->lflag && strcmp(a + 2, s->lflag) == 0);
                if (!hit) continue;
                matched = 1;
                if (s->seen)
                    fail("error: Argument already set! for arg -%s\n\n", s->sflag);
                s->seen = 1;
                if (!s->is_switch) {
                    if (i + 1 >= argc) fail("error: Missing a value for this argument! for arg -%s\n\n", s->sflag);
                    s->value = argv[++i];
                }
            }
            if (!matched && a[1] != '-') {
                /* combined switches, e.g. -qD */
                int all = 1;
                for (const char *c = a + 1; *c && all; ++c) {
                    int f = 0;
                    for (int k = 0; k < nspec; ++k)
                        if (specs[k].is_switch && specs[k].sflag && specs[k].sflag[0] == *c && !specs[k].sflag[1]) f = 1;
                    all = f;
                }
                if (all) {
                    for (const char *c = a + 1; *c; ++c)
                        for (int k = 0; k < nspec; ++k)
                            if (specs[k].is_switch && specs[k].sflag && specs[k].sflag[0] == *c && !specs[k].sflag[1]) specs[k].seen = 1;
                    matched = 1;
                }
            }
            if (!matched) fail("error: Couldn't find match for argument for arg %s\n\n", a);
        } else {
            (*pos)[(*npos)++] = argv[i];
        }
    }
    for (int k = 0; k < nspec; ++k)
        if (specs[k].required && !specs[k].seen)
            fail("error: Required argument missing for arg -%s\n\n", specs[k].sflag);
    return 0;
}

static double arg_double(const argspec *s, double dflt) {
    if (!s->seen) return dflt;
    double v;
    if (!lex_double(s->value, &v)) fail("error: Couldn't read argument value from string '%s' for arg -%s\n\n", s->value, s->sflag);
    return v;
}
static uint64_t arg_uint(const argspec *s, uint64_t dflt, uint64_t maxv) {
    if (!s->seen) return dflt;
    uint64_t v;
    if (!lex_u64(s->value, strlen(s->value), maxv, &v)) fail("error: Couldn't read argument value from string '%s' for arg -%s\n\n", s->value, s->sflag);
    return v;
}

static void parse_offsets(const char *str, int nfiles, short **offs, int *noffs) {
    *noffs = 0;
    *offs = NULL;
    if (!str || !*str) return;
    char **tok;
    int n = split_csv(str, &tok);
    *offs = (short *)xcalloc((size_t)n, sizeof(short));
    for (int i = 0; i < n; ++i)
        if (!lex_short(tok[i], &(*offs)[i])) fail("error: bad offset argument\n\n");
    if (!(n == nfiles || n == 1))
        fail("error: wrong number of offset arguments\nmust have same number as alignment files or just one\n\n");
    *noffs = n;
}

/* ---------------------------------------------------------------------- */
/* bin/regions -- src/regions.cpp:27-409                                    */
/* ---------------------------------------------------------------------- */
typedef struct {
    orc_region **v;
    size_t n, cap;
} regvec;

static void regvec_push(void *user, orc_region *g) {
    regvec *rv = (regvec *)user;
    if (rv->n == rv->cap) {
        rv->cap = rv->cap ? rv->cap * 2 : 64;
        rv->v = (orc_region **)realloc(rv->v, rv->cap * sizeof(orc_region *));
    }
    rv->v[rv->n++] = g;
}

typedef struct {
    FILE *fp;
    const ctab *ct;
    int peaks, corrs;
} region_writer;

/* FormatOutStream::write(const Region&), format.cpp:1141-1162 */
static void write_region(region_writer *w, const orc_region *g, uint16_t n_expt) {
    sbuf b = {0};
    const uint64_t left = orc_region_left(g);
    const uint64_t right = left + orc_region_npos(g) - 1;
    sb_printf(&b, "%s:", w->ct->names[orc_region_contig(g)]);
    if (orc_region_forward(g)) sb_printf(&b, "%llu-%llu", (unsigned long long)left, (unsigned long long)right);
    else sb_printf(&b, "%llu-%llu", (unsigned long long)right, (unsigned long long)left);
    if (w->peaks) sb_printf(&b, "\t%u", orc_region_peak(g));
    if (w->corrs) {
        sb_puts(&b, "\t");
        sb_os(&b, orc_region_corr(g, 0));
    }
    sb_printf(&b, "\t%.2f", orc_region_kurtosis(g));
    uint32_t *sums = (uint32_t *)xcalloc(n_expt, sizeof(uint32_t));
    orc_region_expt_sums(g, sums);
    for (uint16_t s = 0; s < n_expt; ++s) sb_printf(&b, "\t%u", sums[s]);
    sb_puts(&b, "\n");
    fwrite(b.p, 1, b.n, w->fp);
    free(sums);
    free(b.p);
}

static FILE *open_out(const char *fname) {
    if (strcmp(fname, "stdout") == 0) return stdout;
    FILE *fp = filter_open(fname, 1);
    if (!fp) fail("error: could not write %s\n\n", fname);
    return fp;
}

/* density profile writer: FormatOutStream::write(const PosScore&) and
 * trackHeader(), misc/format.cpp:1091-1132, 1164-1219; constants
 * misc/defaults.hpp:38-42 (colours, PROFILE_PRIORITY = 2) */
typedef struct {
    FILE *fp;
    const ctab *ct;
    int directional;
    const char *name, *assembly;
    int have_contig, forward;
    uint32_t contig;
} prof_writer;

static void prof_track_header(prof_writer *w) {
    fprintf(w->fp, "track name=\"%s", w->name);
    if (w->directional) fputs(w->forward ? " +" : " -", w->fp);
    fputc('"', w->fp);
    if (w->directional) fprintf(w->fp, " description=\"%s\"", w->forward ? w->name : " ");
    fputs(" priority=2 visibility=", w->fp);
    if (w->directional)
        fputs(w->forward ? "full type=wiggle_0 alwaysZero=on color=0,0,255"
                         : "full type=wiggle_0 alwaysZero=on color=255,0,0 altColor=255,0,0", w->fp);
    else
        fputs("full type=wiggle_0 alwaysZero=on color=191,0,191", w->fp);
    if (*w->assembly) fprintf(w->fp, " db=%s", w->assembly);
    fputc('\n', w->fp);
}

static void prof_write(void *user, int forward, uint32_t contig, uint32_t pos, double score) {
    prof_writer *w = (prof_writer *)user;
    if (score == 0) return;
    if (w->directional) {
        if (!w->have_contig || w->forward != forward) {
            w->forward = forward;
            w->have_contig = 0;
            prof_track_header(w);
        }
    } else if (!w->have_contig) {
        prof_track_header(w);
    }
    if (!w->have_contig || w->contig != contig) {  /* names are unique in the table */
        w->contig = contig;
        w->have_contig = 1;
        fprintf(w->fp, "variableStep chrom=%s\n", w->ct->names[contig]);
    }
    fprintf(w->fp, "%u ", pos);
    if (w->directional && !forward) fputc('-', w->fp);
    fprintf(w->fp, "%g\n", score);
}

int orc_regions_main(int argc, char **argv) {
    argspec sp[] = {
        {"q", "quiet", 1, 0, 0, 0},          {"D", "non-directional", 1, 0, 0, 0},
        {"a", "assembly", 0, 0, 0, 0},       {"n", "name", 0, 0, 0, 0},
        {"w", "wig", 0, 0, 0, 0},            {"m", "mappable", 0, 0, 0, 0},
        {"t", "hitThreshold", 0, 0, 0, 0},   {"y", "corr", 1, 0, 0, 0},
        {"u", "corrThreshold", 0, 0, 0, 0},  {"k", "kurtosisThreshold", 0, 0, 0, 0},
        {"r", "regionThreshold", 0, 0, 0, 0}, {"z", "coeff", 0, 0, 0, 0},
        {"b", "bandwidth", 0, 0, 0, 0},      {"i", "mismatches", 0, 0, 0, 0},
        {"l", "length", 0, 0, 0, 0},         {"s", "shift", 0, 0, 0, 0},
        {"p", "prob", 0, 0, 0, 0},           {"e", "exclude", 0, 0, 0, 0},
        {"f", "peaks", 1, 0, 0, 0},          {"o", "out", 0, 1, 0, 0},
        {"c", "contig", 0, 1, 0, 0},
    };
    const int nsp = (int)(sizeof sp / sizeof sp[0]);
    char **files;
    int nfiles;
    parse_args(argc, argv, sp, nsp, &files, &nfiles);
    if (nfiles == 0) fail("error: Required argument missing for arg alignment filenames\n\n");
    const int quiet = sp[0].seen, directional = !sp[1].seen;
    const char *profile = sp[4].seen ? sp[4].value : "";
    const char *assembly = sp[2].seen ? sp[2].value : "";
    const char *track_nm = sp[3].seen ? sp[3].value : "";
    uint32_t mappable = (uint32_t)arg_uint(&sp[5], 0, 0xFFFFFFFFull);
    double hit_thr = arg_double(&sp[6], 10);
    int out_corrs = sp[7].seen;
    double corr_thr = arg_double(&sp[8], 0.3);
    double kurt_thr = arg_double(&sp[9], 50);
    double region_thr = arg_double(&sp[10], 25);
    const char *coeff_str = sp[11].seen ? sp[11].value : "";
    uint16_t bw = (uint16_t)arg_uint(&sp[12], 50, 0xFFFF);
    uint16_t use_len = (uint16_t)arg_uint(&sp[14], 0, 0xFFFF);
    const char *offset_str = sp[15].seen ? sp[15].value : "";
    const char *control_str = sp[17].seen ? sp[17].value : "";
    int out_peaks = sp[18].seen;
    const char *out_name = sp[19].value;
    const char *ct_name = sp[20].value;

    if (directional) {
        if (corr_thr != 0.3) fprintf(stderr, "warning: correlation threshold is not used on strand-specific analysis\n");
        corr_thr = -1;
        if (out_corrs) fprintf(stderr, "warning: strand correlations are not calculated for strand-specific analysis\n");
        out_corrs = 0;
    }
    short *offs;
    int noffs;
    parse_offsets(offset_str, nfiles, &offs, &noffs);

    uint8_t *control = (uint8_t *)xcalloc((size_t)nfiles, 1);
    if (*control_str) {
        char **tok;
        int n = split_csv(control_str, &tok);
        for (int i = 0; i < n; ++i) {
            short v;
            if (!lex_short(tok[i], &v)) fail("error: bad control index\n\n");
            uint16_t idx = (uint16_t)v;
            if (idx == 0) fail("error: bad control index (first sample is 1)\n\n");
            if (idx > nfiles) fail("error: bad control index (greater than number of samples)\n\n");
            control[idx - 1] = 1;
        }
    }
    uint16_t n_control = 0;
    for (int i = 0; i < nfiles; ++i) n_control += control[i];
    hit_thr *= (double)(nfiles - n_control);

    double *coeffs = (double *)xcalloc((size_t)nfiles + 1, sizeof(double));
    int ncoeffs = 0, prop_coeffs = 0;
    if (*coeff_str) {
        if (strcmp(coeff_str, "p") == 0) {
            prop_coeffs = 1;
        } else {
            char **tok;
            int n = split_csv(coeff_str, &tok);
            coeffs = (double *)realloc(coeffs, ((size_t)n + 1) * sizeof(double));
            for (int i = 0; i < n; ++i)
                if (!lex_double(tok[i], &coeffs[i])) fail("error: bad coeff argument\n\n");
            ncoeffs = n;
            if (ncoeffs != nfiles - n_control)
                fail("error: wrong number of coeff arguments\nmust have same number as non-control alignment files\n\n");
        }
    }

    ctab *ct = ctab_parse(ct_name);

    stream_t *st = (stream_t *)xcalloc((size_t)nfiles, sizeof(stream_t));
    uint64_t non_control_tags = 0, total_tags = 0;
    fprintf(stderr, "reading alignment files...\n");
    for (int i = 0, oi = 0; i < nfiles; ++i) {
        const short off = noffs ? offs[oi] : 0;
        st_open(&st[i], files[i], ct, off, use_len, !directional);
        const uint64_t tags = st_expected(&st[i]);
        if (!control[i]) non_control_tags += tags;
        total_tags += tags;
        st_read(&st[i]);
        fprintf(stderr, "  %s: %llu tags\n", st_name(&st[i]), (unsigned long long)tags);
        if (noffs > 1) ++oi;
    }
    if (mappable == 0) mappable = ct->genome;
    fprintf(stderr, "%llu usable tags", (unsigned long long)total_tags);
    if (non_control_tags != total_tags) fprintf(stderr, ", %llu not from negative controls,", (unsigned long long)non_control_tags);
    fprintf(stderr, " at %u mappable positions\n", mappable);
    double background = (double)non_control_tags / (double)mappable;
    if (directional) background /= 2;
    fprintf(stderr, "using background = %g tags/position%s\n", background, directional ? " on each strand" : "");

    if (prop_coeffs) {
        for (int i = 0; i < nfiles; ++i)
            if (!control[i])
                coeffs[ncoeffs++] = (double)non_control_tags / ((double)st_expected(&st[i]) * (double)(nfiles - n_control));
    } else if (ncoeffs) {
        /* Q6: the coefficient iterator advances with every sample */
        double scaled = 0;
        for (int i = 0, j = 0; i < ncoeffs && j < nfiles; ++i, ++j)
            if (!control[j]) scaled += coeffs[i] * (double)st_expected(&st[j]);
        for (int i = 0; i < ncoeffs; ++i) coeffs[i] *= (double)non_control_tags / scaled;
    }

    const uint32_t W = 2u * bw + 1;
    double *kern = (double *)xcalloc(W, sizeof(double));
    orc_kernel(bw, 1 / background, kern);

    sbuf hdr = {0};
    for (int i = 0; i < nfiles; ++i) sb_printf(&hdr, "# align_file=%s\n", files[i]);
    if (noffs) {
        if (noffs == 1) sb_printf(&hdr, "# shift=%d\n", offs[0]);
        else {
            sb_puts(&hdr, "# shifts=");
            for (int i = 0; i < noffs - 1; ++i) sb_printf(&hdr, "%d,", offs[i]);
            sb_printf(&hdr, "%d\n", offs[noffs - 1]);
        }
    }
    sb_printf(&hdr, "# contig_table=%s\n", ct_name);
    sb_printf(&hdr, "# bandwidth=%u\n", bw);
    if (nfiles > 1) {
        sb_printf(&hdr, "# tags=%llu", (unsigned long long)st_expected(&st[0]));
        for (int i = 1; i < nfiles; ++i) sb_printf(&hdr, ",%llu", (unsigned long long)st_expected(&st[i]));
        sb_puts(&hdr, "\n");
    }
    if (n_control > 0) {
        sb_puts(&hdr, "# control=");
        int first = 1;
        for (int i = 0; i < nfiles; ++i)
            if (control[i]) {
                if (!first) sb_puts(&hdr, ",");
                first = 0;
                sb_printf(&hdr, "%d", i + 1);
            }
        sb_puts(&hdr, "\n");
    }
    if (ncoeffs) {
        sb_puts(&hdr, "# coeffs=");
        sb_os(&hdr, coeffs[0]);
        for (int i = 1; i < ncoeffs; ++i) { sb_puts(&hdr, ","); sb_os(&hdr, coeffs[i]); }
        sb_puts(&hdr, "\n");
    }
    sb_printf(&hdr, "# total_tags=%llu\n", (unsigned long long)non_control_tags);
    sb_puts(&hdr, "# background=");
    sb_os(&hdr, background);
    sb_puts(&hdr, "\n");

    /* regions.cpp:103, 276-284: the profile stream gets the common header */
    prof_writer pw = {0};
    if (*profile) {
        pw.fp = open_out(profile);
        pw.ct = ct;
        pw.directional = directional;
        pw.name = *track_nm ? track_nm : fname_prefix(profile);
        pw.assembly = assembly;
        fwrite(hdr.p, 1, hdr.n, pw.fp);
    }
    FILE *out = open_out(out_name);
    region_writer wr = {out, ct, out_peaks, out_corrs};
    fwrite(hdr.p, 1, hdr.n, out);
    sbuf h2 = {0};
    sb_puts(&h2, "# region_threshold="); sb_lex(&h2, region_thr); sb_puts(&h2, "\n");
    sb_puts(&h2, "# kurtosis_threshold="); sb_lex(&h2, kurt_thr); sb_puts(&h2, "\n");
    sb_puts(&h2, "# corr_threshold="); sb_lex(&h2, corr_thr); sb_puts(&h2, "\n");
    sb_puts(&h2, "# hit_threshold="); sb_lex(&h2, hit_thr); sb_puts(&h2, "\n");
    if (out_peaks) sb_puts(&h2, "\tpeak");
    if (out_corrs) sb_puts(&h2, "\tcorrelation");
    sb_puts(&h2, "\tkurtosis");
    for (int i = 0; i < nfiles; ++i) sb_printf(&h2, "\t%s", st_name(&st[i]));
    sb_puts(&h2, "\n");
    fwrite(h2.p, 1, h2.n, out);

    fprintf(stderr, "calling enriched regions...\n");
    regvec pending = {0};
    orc_buf *fb = orc_buf_new(kern, W, region_thr, kurt_thr, corr_thr, hit_thr, 1,
                              (uint16_t)nfiles, control, coeffs, (uint32_t)ncoeffs,
                              regvec_push, &pending, *profile ? prof_write : NULL, &pw);
    orc_buf *rb = orc_buf_new(kern, W, region_thr, kurt_thr, corr_thr, hit_thr, 0,
                              (uint16_t)nfiles, control, coeffs, (uint32_t)ncoeffs,
                              regvec_push, &pending, *profile ? prof_write : NULL, &pw);
    uint32_t *fh = (uint32_t *)xcalloc((size_t)nfiles, sizeof(uint32_t));
    uint32_t *rh = (uint32_t *)xcalloc((size_t)nfiles, sizeof(uint32_t));
    uint32_t contig = 0;
    int forward = 1;
    while (contig < ct->n) {
        if (!quiet) fprintf(stderr, "  %s%s... ", ct->names[contig], directional ? (forward ? "+" : "-") : "");
        const uint32_t lim = ct->sizes[contig];
        uint32_t pos = 1;
        while (pos <= lim) {
            int ff = 0, fr = 0;
            uint32_t next = lim + 1;
            for (int i = 0; i < nfiles; ++i) {
                fh[i] = 0;
                rh[i] = 0;
                const align_t *a = st_last(&st[i]);
                while (a->count != 0 && a->first == pos && a->contig == contig) {
                    if (a->forward) { fh[i] += a->count; ff = 1; }
                    else { rh[i] += a->count; fr = 1; }
                    a = st_read(&st[i]);
                }
                if (a->count != 0 && a->contig == contig && a->first < next) next = a->first;
            }
            if (ff) orc_buf_add(fb, fh, contig, pos, 1);
            if (fr) {
                if (directional) orc_buf_add(rb, rh, contig, pos, 0);
                else orc_buf_add(fb, rh, contig, pos, 0);
            }
            if (pending.n) {
                for (size_t k = 0; k < pending.n; ++k) {
                    write_region(&wr, pending.v[k], (uint16_t)nfiles);
                    orc_region_free(pending.v[k]);
                }
                pending.n = 0;
            }
            pos = next;
        }
        const uint64_t fr_n = orc_buf_flush(fb);
        const uint64_t rr_n = orc_buf_flush(rb);
        if (!quiet) {
            if (forward) {
                fprintf(stderr, "%llu\n", (unsigned long long)fr_n);
                if (directional && rr_n > 0) fprintf(stderr, "  %s-... %llu\n", ct->names[contig], (unsigned long long)rr_n);
            } else {
                fprintf(stderr, "%llu\n", (unsigned long long)rr_n);
            }
        }
        ++contig;
        if (directional && contig == ct->n && forward) {
            contig = 0;
            forward = 0;
        }
    }
    if (out != stdout) fclose(out); else fflush(out);
    if (pw.fp) { if (pw.fp != stdout) fclose(pw.fp); else fflush(pw.fp); }
    /* Q3: regions closed by the final flush are never written */
    for (size_t k = 0; k < pending.n; ++k) orc_region_free(pending.v[k]);

    fprintf(stderr, "%llu regions passed filters, %llu rejected\n",
            (unsigned long long)(orc_buf_nregions(fb) + orc_buf_nregions(rb)),
            (unsigned long long)(orc_buf_nrejects(fb) + orc_buf_nrejects(rb)));
    fprintf(stderr, "tags in regions:\n");
    for (int i = 0; i < nfiles; ++i) {
        const uint64_t conf = st_confident(&st[i]);
        if (conf + st_oob(&st[i]) != st_expected(&st[i]))
            fprintf(stderr, "  warning: expected %llu tags in %s but found %llu; results inaccurate\n",
                    (unsigned long long)st_expected(&st[i]), st_name(&st[i]), (unsigned long long)conf);
        const uint64_t tir = orc_buf_tags_in_regions(fb)[i] + orc_buf_tags_in_regions(rb)[i];
        fprintf(stderr, "  %s: %llu (%.1f%%)\n", st_name(&st[i]), (unsigned long long)tir,
                100 * (double)tir / (double)conf);
    }
    fprintf(stderr, "\nAll done!\n\n");
    orc_buf_free(fb);
    orc_buf_free(rb);
    return 0;
}

/* ---------------------------------------------------------------------- */
/* libstdc++ std::sort (introsort) restated for Q15 tie order              */
/* ---------------------------------------------------------------------- */
typedef struct {
    orc_region *g;
    uint32_t sum;
} sortrec;

static int cmp_gt(const sortrec *a, const sortrec *b) { return a->sum > b->sum; }

static void sr_swap(sortrec *a, sortrec *b) {
    sortrec t = *a;
    *a = *b;
    *b = t;
}

static void move_median_to_first(sortrec *result, sortrec *a, sortrec *b, sortrec *c) {
    if (cmp_gt(a, b)) {
        if (cmp_gt(b, c)) sr_swap(result, b);
        else if (cmp_gt(a, c)) sr_swap(result, c);
        else sr_swap(result, a);
    } else if (cmp_gt(a, c)) sr_swap(result, a);
    else if (cmp_gt(b, c)) sr_swap(result, c);
    else sr_swap(result, b);
}

static sortrec *unguarded_partition(sortrec *first, sortrec *last, sortrec *pivot) {
    while (1) {
        while (cmp_gt(first, pivot)) ++first;
        --last;
        while (cmp_gt(pivot, last)) --last;
        if (!(first < last)) return first;
        sr_swap(first, last);
        ++first;
    }
}

static void adjust_heap(sortrec *first, ptrdiff_t hole, ptrdiff_t len, sortrec value) {
    const ptrdiff_t top = hole;
    ptrdiff_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (cmp_gt(&first[child], &first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    ptrdiff_t parent = (hole - 1) / 2;
    while (hole > top && cmp_gt(&first[parent], &value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

static void heap_select_sort(sortrec *first, sortrec *last) {
    const ptrdiff_t len = last - first;
    if (len >= 2)
        for (ptrdiff_t parent = (len - 2) / 2;; --parent) {
            adjust_heap(first, parent, len, first[parent]);
            if (parent == 0) break;
        }
    while (last - first > 1) {
        --last;
        sortrec v = *last;
        *last = *first;
        adjust_heap(first, 0, last - first, v);
    }
}

static void introsort_loop(sortrec *first, sortrec *last, long depth) {
    while (last - first > 16) {
        if (depth == 0) {
            heap_select_sort(first, last);
            return;
        }
        --depth;
        sortrec *mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1);
        sortrec *cut = unguarded_partition(first + 1, last, first);
        introsort_loop(cut, last, depth);
        last = cut;
    }
}

static void insertion_sort(sortrec *first, sortrec *last) {
    if (first == last) return;
    for (sortrec *i = first + 1; i != last; ++i) {
        if (cmp_gt(i, first)) {
            sortrec v = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(sortrec));
            *first = v;
        } else {
            sortrec v = *i;
            sortrec *j = i, *k = i - 1;
            while (cmp_gt(&v, k)) { *j = *k; j = k; --k; }
            *j = v;
        }
    }
}

static void unguarded_insertion_sort(sortrec *first, sortrec *last) {
    for (sortrec *i = first; i != last; ++i) {
        sortrec v = *i;
        sortrec *j = i, *k = i - 1;
        while (cmp_gt(&v, k)) { *j = *k; j = k; --k; }
        *j = v;
    }
}

static void std_sort(sortrec *first, sortrec *last) {
    if (first == last) return;
    long n = (long)(last - first), lg = 0;
    while (n > 1) { n >>= 1; ++lg; }
    introsort_loop(first, last, 2 * lg);
    if (last - first > 16) {
        insertion_sort(first, first + 16);
        unguarded_insertion_sort(first + 16, last);
    } else {
        insertion_sort(first, last);
    }
}

/* ---------------------------------------------------------------------- */
/* bin/strand_shift -- src/strand_shift.cpp:31-304                          */
/* ---------------------------------------------------------------------- */
int orc_strand_shift_main(int argc, char **argv) {
    argspec sp[] = {
        {"m", "mappable", 0, 0, 0, 0},       {"t", "hitThreshold", 0, 0, 0, 0},
        {"u", "corrThreshold", 0, 0, 0, 0},  {"k", "kurtosisThreshold", 0, 0, 0, 0},
        {"r", "regionThreshold", 0, 0, 0, 0}, {"b", "bandwidth", 0, 0, 0, 0},
        {"g", "testRegions", 0, 0, 0, 0},    {"x", "maxShift", 0, 0, 0, 0},
        {"n", "minShift", 0, 0, 0, 0},       {"i", "mismatches", 0, 0, 0, 0},
        {"l", "length", 0, 0, 0, 0},         {"s", "shift", 0, 0, 0, 0},
        {"p", "prob", 0, 0, 0, 0},           {"o", "out", 0, 0, 0, 0},
        {"c", "contigs", 0, 1, 0, 0},
    };
    const int nsp = (int)(sizeof sp / sizeof sp[0]);
    char **files;
    int nfiles;
    parse_args(argc, argv, sp, nsp, &files, &nfiles);
    if (nfiles == 0) fail("error: Required argument missing for arg alignment filenames\n\n");
    uint32_t mappable = (uint32_t)arg_uint(&sp[0], 0, 0xFFFFFFFFull);
    uint32_t hit_thr = (uint32_t)arg_uint(&sp[1], 10, 0xFFFFFFFFull);
    double corr_thr = arg_double(&sp[2], 0.3);
    double kurt_thr = arg_double(&sp[3], 50);
    double region_thr = arg_double(&sp[4], 25);
    uint16_t bw = (uint16_t)arg_uint(&sp[5], 50, 0xFFFF);
    uint16_t n_test = (uint16_t)arg_uint(&sp[6], 1000, 0xFFFF);
    uint16_t max_shift = (uint16_t)arg_uint(&sp[7], 150, 0xFFFF);
    uint16_t min_shift = (uint16_t)arg_uint(&sp[8], 25, 0xFFFF);
    uint16_t use_len = (uint16_t)arg_uint(&sp[10], 0, 0xFFFF);
    const char *offset_str = sp[11].seen ? sp[11].value : "";
    const char *out_name = sp[13].seen ? sp[13].value : "";
    const char *ct_name = sp[14].value;

    short *offs;
    int noffs;
    parse_offsets(offset_str, nfiles, &offs, &noffs);
    ctab *ct = ctab_parse(ct_name);
    stream_t *st = (stream_t *)xcalloc((size_t)nfiles, sizeof(stream_t));
    uint64_t total = 0;
    fprintf(stderr, "reading alignment files...\n");
    for (int i = 0, oi = 0; i < nfiles; ++i) {
        const short off = noffs ? offs[oi] : 0;
        st_open(&st[i], files[i], ct, off, use_len, 1);
        const uint64_t tags = st_expected(&st[i]);
        total += tags;
        st_read(&st[i]);
        fprintf(stderr, "  %s: %llu tags\n", st_name(&st[i]), (unsigned long long)tags);
        if (noffs > 1) ++oi;
    }
    if (mappable == 0) mappable = ct->genome;
    fprintf(stderr, "%llu usable tags at %u mappable positions\n", (unsigned long long)total, mappable);
    const double background = (double)total / (double)mappable;
    fprintf(stderr, "using background = %g tags/position\n", background);
    const uint32_t W = 2u * bw + 1;
    double *kern = (double *)xcalloc(W, sizeof(double));
    orc_kernel(bw, 1 / background, kern);

    fprintf(stderr, "calling enriched regions for shift calibration... ");
    regvec regs = {0};
    uint8_t *control = (uint8_t *)xcalloc((size_t)nfiles, 1);
    orc_buf *b = orc_buf_new(kern, W, region_thr, kurt_thr, -1, (double)hit_thr, 1,
                             (uint16_t)nfiles, control, NULL, 0, regvec_push, &regs, NULL, NULL);
    uint32_t *fh = (uint32_t *)xcalloc((size_t)nfiles, sizeof(uint32_t));
    uint32_t *rh = (uint32_t *)xcalloc((size_t)nfiles, sizeof(uint32_t));
    for (uint32_t contig = 0; contig < ct->n; ++contig) {
        const uint32_t lim = ct->sizes[contig];
        uint32_t pos = 1;
        while (pos <= lim) {
            int ff = 0, fr = 0;
            uint32_t next = lim + 1;
            for (int i = 0; i < nfiles; ++i) {
                fh[i] = 0;
                rh[i] = 0;
                const align_t *a = st_last(&st[i]);
                while (a->count != 0 && a->first == pos && a->contig == contig) {
                    if (a->forward) { fh[i] += a->count; ff = 1; }
                    else { rh[i] += a->count; fr = 1; }
                    a = st_read(&st[i]);
                }
                if (a->count != 0 && a->contig == contig && a->first < next) next = a->first;
            }
            if (ff) orc_buf_add(b, fh, contig, pos, 1);
            if (fr) orc_buf_add(b, rh, contig, pos, 0);
            pos = next;
        }
        orc_buf_flush(b);
    }
    fprintf(stderr, "%zu found\n", regs.n);

    sortrec *sr = (sortrec *)xcalloc(regs.n, sizeof(sortrec));
    for (size_t i = 0; i < regs.n; ++i) {
        sr[i].g = regs.v[i];
        sr[i].sum = orc_region_sum(regs.v[i]);
    }
    std_sort(sr, sr + regs.n);

    uint16_t tested = 0;
    uint64_t tags_in = 0;
    uint64_t *freq = (uint64_t *)xcalloc((size_t)max_shift + 1, sizeof(uint64_t));
    for (size_t i = 0; tested < n_test && i < regs.n; ++i) {
        const orc_region *g = sr[i].g;
        if (orc_region_npos(g) > (unsigned)(2 * max_shift + 3)) {
            uint16_t best = 0;
            double best_corr = -1;
            for (uint16_t s = 0; s <= max_shift; ++s) {
                const double c = orc_region_corr(g, s);
                if (c > best_corr) { best = s; best_corr = c; }
                if (s == 0xFFFF) break;
            }
            if (best_corr >= corr_thr) {
                ++freq[best];
                tags_in += sr[i].sum;
                ++tested;
            }
        }
    }
    if (tested == 0) fail("error: no regions qualified with given settings\n\n");
    if (tested < n_test) fprintf(stderr, "warning: too few regions qualified with given settings\n");
    fprintf(stderr, "the top %u qualified regions contained %llu tags (%.1f%%)\n", tested,
            (unsigned long long)tags_in, 100 * (double)tags_in / (double)total);

    double mk[11];
    orc_kernel(5, 1, mk);
    const size_t nd = (size_t)max_shift + 1;
    double *dens = (double *)xcalloc(nd, sizeof(double));
    for (uint16_t i = 0; i < nd; ++i)
        for (int j = 0; j < 11; ++j) {
            const int k = (int)i - 5 + j;
            if (k >= 0 && k < (int)nd) dens[k] += (double)freq[i] * mk[j];
        }
    double best_d = 0;
    uint16_t best_shift = 0;
    for (uint16_t i = min_shift; i < nd - 5; ++i)
        if (dens[i] > best_d) { best_shift = i; best_d = dens[i]; }
    fprintf(stderr, "estimated shift = %u\n", best_shift);

    if (*out_name) {
        fprintf(stderr, "writing output to %s... ", out_name);
        FILE *out = open_out(out_name);
        sbuf o = {0};
        for (int i = 0; i < nfiles; ++i) sb_printf(&o, "# align_file=%s\n", files[i]);
        if (noffs) {
            if (noffs == 1) { sb_puts(&o, "# shift="); sb_lex(&o, offs[0]); sb_puts(&o, "\n"); }
            else {
                sb_puts(&o, "# shifts=");
                for (int i = 0; i < noffs - 1; ++i) { sb_lex(&o, offs[i]); sb_puts(&o, ","); }
                sb_lex(&o, offs[noffs - 1]);
                sb_puts(&o, "\n");
            }
        }
        sb_printf(&o, "# contig_table=%s\n", ct_name);
        sb_puts(&o, "# bandwidth="); sb_lex(&o, bw); sb_puts(&o, "\n");
        sb_puts(&o, "# tags="); sb_lex(&o, (double)total); sb_puts(&o, "\n");
        sb_puts(&o, "# background="); sb_lex(&o, background); sb_puts(&o, "\n");
        sb_puts(&o, "# region_threshold="); sb_lex(&o, region_thr); sb_puts(&o, "\n");
        sb_puts(&o, "# kurtosis_threshold="); sb_lex(&o, kurt_thr); sb_puts(&o, "\n");
        sb_puts(&o, "# corr_threshold="); sb_lex(&o, corr_thr); sb_puts(&o, "\n");
        sb_puts(&o, "# hit_threshold="); sb_lex(&o, hit_thr); sb_puts(&o, "\n");
        sb_puts(&o, "# regions_tested="); sb_lex(&o, tested); sb_puts(&o, "\n");
        sb_puts(&o, "# tags_in_regions="); sb_lex(&o, (double)tags_in); sb_puts(&o, "\n");
        sb_puts(&o, "# min_shift="); sb_lex(&o, min_shift); sb_puts(&o, "\n");
        sb_puts(&o, "# best_shift="); sb_lex(&o, best_shift); sb_puts(&o, "\n\n");
        sb_puts(&o, "shift\tregions\n");
        for (uint16_t i = 0; i < nd; ++i)
            if (freq[i]) {
                sb_lex(&o, i);
                sb_puts(&o, "\t");
                sb_lex(&o, (double)freq[i]);
                sb_puts(&o, "\n");
            }
        fwrite(o.p, 1, o.n, out);
        if (out != stdout) fclose(out); else fflush(out);
    }
    fprintf(stderr, "done!\n\n");
    for (size_t i = 0; i < regs.n; ++i) orc_region_free(regs.v[i]);
    orc_buf_free(b);
    return 0;
}

/* ---------------------------------------------------------------------- */
/* bin/tags_in_regions -- src/tags_in_regions.cpp:22-214                    */
/* ---------------------------------------------------------------------- */
int orc_tags_in_regions_main(int argc, char **argv) {
    argspec sp[] = {
        {"D", "non-directional", 1, 0, 0, 0}, {"i", "mismatches", 0, 0, 0, 0},
        {"l", "length", 0, 0, 0, 0},          {"s", "shift", 0, 0, 0, 0},
        {"p", "prob", 0, 0, 0, 0},            {"e", "extend", 0, 0, 0, 0},
        {"o", "out", 0, 1, 0, 0},             {"f", "in", 0, 1, 0, 0},
        {"c", "contig", 0, 1, 0, 0},
    };
    const int nsp = (int)(sizeof sp / sizeof sp[0]);
    char **files;
    int nfiles;
    parse_args(argc, argv, sp, nsp, &files, &nfiles);
    if (nfiles == 0) fail("error: Required argument missing for arg alignment filenames\n\n");
    const int directional = !sp[0].seen;
    uint16_t use_len = (uint16_t)arg_uint(&sp[2], 0, 0xFFFF);
    const char *offset_str = sp[3].seen ? sp[3].value : "";
    uint32_t ext = (uint32_t)arg_uint(&sp[5], 0, 0xFFFFFFFFull);
    const char *out_name = sp[6].value, *in_name = sp[7].value, *ct_name = sp[8].value;

    short *offs;
    int noffs;
    parse_offsets(offset_str, nfiles, &offs, &noffs);
    ctab *ct = ctab_parse(ct_name);
    stream_t *st = (stream_t *)xcalloc((size_t)nfiles, sizeof(stream_t));
    fprintf(stderr, "reading alignment files...\n");
    for (int i = 0, oi = 0; i < nfiles; ++i) {
        const short off = noffs ? offs[oi] : 0;
        st_open(&st[i], files[i], ct, off, use_len, !directional);
        const uint64_t tags = st_expected(&st[i]);
        st_read(&st[i]);
        fprintf(stderr, "  %s: %llu tags\n", st_name(&st[i]), (unsigned long long)tags);
        if (noffs > 1) ++oi;
    }
    instream rin;
    in_open(&rin, in_name);
    FILE *out = open_out(out_name);
    sbuf o = {0};
    size_t len;
    const char *l = in_read_line(&rin, &len);
    char *line = (char *)xcalloc(len + 1, 1);
    memcpy(line, l, len);
    while (len == 0 || line[0] == '#') {
        sb_printf(&o, "%s\n", line);
        l = in_read_line(&rin, &len);
        free(line);
        line = (char *)xcalloc(len + 1, 1);
        memcpy(line, l, len);
    }
    if (line[0] != '\t')
        fail("error: bad format in %s line %llu\n\n", in_name, (unsigned long long)rin.line_no);
    if (ext != 0) { sb_puts(&o, "# region_extension="); sb_lex(&o, ext); sb_puts(&o, "\n"); }
    for (int i = 0; i < nfiles; ++i) sb_printf(&o, "# extra_align_file=%s\n", files[i]);
    if (noffs) {
        if (noffs == 1) { sb_puts(&o, "# shift="); sb_lex(&o, offs[0]); sb_puts(&o, "\n"); }
        else {
            sb_puts(&o, "# shifts=");
            for (int i = 0; i < noffs - 1; ++i) { sb_lex(&o, offs[i]); sb_puts(&o, ","); }
            sb_lex(&o, offs[noffs - 1]);
            sb_puts(&o, "\n");
        }
    }
    sb_puts(&o, line);
    for (int i = 0; i < nfiles; ++i) sb_printf(&o, "\t%s", st_name(&st[i]));
    sb_puts(&o, "\n");
    fprintf(stderr, "processing regions... ");
    uint64_t *tir = (uint64_t *)xcalloc((size_t)nfiles, sizeof(uint64_t));
    uint64_t nreg = 0;
    uint32_t last_contig = ct->n, last_right = 0;
    while (in_good(&rin)) {
        l = in_read_line(&rin, &len);
        if (len == 0) continue;
        char *ln = (char *)xcalloc(len + 1, 1);
        memcpy(ln, l, len);
        const char *colon = strchr(ln, ':'), *dash = strchr(ln, '-'), *tab = strchr(ln, '\t');
        if (!tab || !colon || !dash || dash > tab || colon > dash)
            fail("error: bad format in %s line %llu\n\n", in_name, (unsigned long long)rin.line_no);
        const uint32_t contig = ctab_find(ct, ln, (size_t)(colon - ln));
        if (contig == ct->n)
            fail("error: contig not in table in %s line %llu\n\n", in_name, (unsigned long long)rin.line_no);
        uint64_t start, end;
        if (!lex_u64(colon + 1, (size_t)(dash - colon - 1), 0xFFFFFFFFull, &start) ||
            !lex_u64(dash + 1, (size_t)(tab - dash - 1), 0xFFFFFFFFull, &end))
            fail("error: bad format in %s line %llu\n\n", in_name, (unsigned long long)rin.line_no);
        const int fwd = end >= start;
        if (!fwd && !directional) fail("error: reverse regions in non-directional analysis\n\n");
        const uint32_t lo = (uint32_t)(fwd ? start : end), hi = (uint32_t)(fwd ? end : start);
        const uint32_t left = lo < ext ? 0 : lo - ext;
        const uint32_t right = hi + ext;
        if (contig == last_contig && left <= last_right) {
            fprintf(stderr, "error: %.*s overlaps previous region", (int)(tab - ln), ln);
            if (ext != 0) fprintf(stderr, "; decrease extension");
            fail("\n\n");
        }
        sb_puts(&o, ln);
        for (int i = 0; i < nfiles; ++i) {
            const align_t *a = st_last(&st[i]);
            while (a->count != 0 && (fwd != a->forward || a->contig < contig || (a->contig == contig && a->first < left)))
                a = st_read(&st[i]);
            uint32_t hits = 0;
            while (a->contig == contig && a->first <= right) {
                hits += a->count;
                a = st_read(&st[i]);
            }
            sb_puts(&o, "\t");
            sb_lex(&o, hits);
            tir[i] += hits;
        }
        sb_puts(&o, "\n");
        ++nreg;
        free(ln);
        /* note: the reference never updates lastContig/lastRight */
    }
    fwrite(o.p, 1, o.n, out);
    if (out != stdout) fclose(out); else fflush(out);
    fprintf(stderr, "%llu in %s\ntags in regions:\n", (unsigned long long)nreg, in_name);
    for (int i = 0; i < nfiles; ++i)
        fprintf(stderr, "  %s: %llu (%.1f%%)\n", st_name(&st[i]), (unsigned long long)tir[i],
                100 * (double)tir[i] / (double)st_expected(&st[i]));
    fprintf(stderr, "\nDone!\n\n");
    return 0;
}
