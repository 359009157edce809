// unipeak_amd/host/wigio.cpp -- see wigio.hpp.
#include "wigio.hpp"
#include "gzio.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <mutex>
#include <thread>

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iostream>

namespace unipeak {

thread_local bool t_defer_errors = false;
void (*g_exit_hook)() = nullptr;

void exit_now(int code) {
    if (g_exit_hook) g_exit_hook();
    std::exit(code);
}

void fatal(const std::string &msg) {
    if (t_defer_errors) throw DeferredError();
    std::cerr << "error: " << msg << "\n" << std::endl;
    exit_now(1);
}

// ---------------------------------------------------------------------------
// number parsing / formatting
// ---------------------------------------------------------------------------
bool lex_uint(const std::string &s, uint64_t maxv, uint64_t *out) {
    size_t i = 0;
    bool neg = false;
    if (s.empty()) return false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i == s.size()) return false;
    uint64_t v = 0;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (maxv - d) / 10) return false;
        v = v * 10 + d;
    }
    if (neg) v = (uint64_t)(0 - v) & maxv;  // lexical_cast<unsigned>("-1") wraps
    *out = v;
    return true;
}

bool lex_short(const std::string &s, int16_t *out) {
    if (s.empty() || std::isspace((unsigned char)s[0])) return false;
    char *e = nullptr;
    errno = 0;
    const long v = std::strtol(s.c_str(), &e, 10);
    if (*e || errno || v < -32768 || v > 32767) return false;
    *out = (int16_t)v;
    return true;
}

bool lex_double(const std::string &s, double *out) {
    if (s.empty() || std::isspace((unsigned char)s[0])) return false;
    char *e = nullptr;
    const double v = std::strtod(s.c_str(), &e);
    if (*e) return false;
    *out = v;
    return true;
}

std::string fmt_lexical(double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}

std::string fmt_ostream(double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%g", v);
    return b;
}

std::string fmt_fixed2(double v) {
    char b[64];
    std::snprintf(b, sizeof b, "%.2f", v);
    return b;
}

std::vector<std::string> split_csv(const std::string &s) {
    std::vector<std::string> out;
    size_t p = 0;
    while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        if (q > p) out.push_back(s.substr(p, q - p));
        p = q + 1;
    }
    return out;
}

std::string fname_prefix(const std::string &path) {
    std::string r = path;
    const size_t sl = r.rfind('/');
    if (sl != std::string::npos) r = r.substr(sl + 1);
    const size_t dot = r.find('.');
    if (dot != std::string::npos) r = r.substr(0, dot);
    return r;
}

// ---------------------------------------------------------------------------
// LexedFile
// ---------------------------------------------------------------------------
unsigned ingest_threads() {
    if (const char *e = std::getenv("UNIPEAK_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) return (unsigned)v;
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min(16u, hw));
}

// canonical data line [p, e): digits, one ' ' or '\t', optional '-', digits
static bool lex_data(const char *p, const char *e, uint32_t *pos, uint32_t *cnt) {
    uint64_t v = 0;
    const char *q = p;
    while (q < e && (unsigned)(*q - '0') < 10u && q - p < 10) v = v * 10 + (uint64_t)(*q++ - '0');
    if (q == p || q == e || (*q != ' ' && *q != '\t') || v > 0xFFFFFFFFull) return false;
    *pos = (uint32_t)v;
    ++q;
    if (q < e && *q == '-') ++q;
    const char *d = q;
    v = 0;
    while (q < e && (unsigned)(*q - '0') < 10u && q - d < 10) v = v * 10 + (uint64_t)(*q++ - '0');
    if (q == d || q != e || v > 0xFFFFFFFFull) return false;
    *cnt = (uint32_t)v;
    return true;
}

LexedFile::~LexedFile() {
    if (base_ && size_ && base_ != inflated_.data()) munmap((void *)base_, size_);
}

void LexedFile::lex(const std::string &fname, int fd, uint64_t size) {
    size_ = size;
    if (size_) {
        void *m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) fatal("could not map " + fname);
        madvise(m, size_, MADV_SEQUENTIAL);
        base_ = (const char *)m;
    }
    lex_bytes();
}

void LexedFile::lex_bytes() {
    // newline-aligned chunk boundaries
    const unsigned T = ingest_threads();
    uint64_t chunk_bytes = 1u << 20;  // UNIPEAK_LEX_CHUNK: tests force many small chunks
    if (const char *e = std::getenv("UNIPEAK_LEX_CHUNK")) chunk_bytes = std::max(1, std::atoi(e));
    uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(4ull * T, size_ / chunk_bytes + 1));
    if (std::getenv("UNIPEAK_LEX_CHUNK")) want = size_ / chunk_bytes + 1;
    std::vector<uint64_t> cut{0};
    for (uint64_t k = 1; k < want; ++k) {
        uint64_t c = size_ * k / want;
        if (c <= cut.back()) continue;
        const void *nl = std::memchr(base_ + c, '\n', size_ - c);
        if (!nl) break;
        c = (uint64_t)((const char *)nl - base_) + 1;
        if (c > cut.back() && c < size_) cut.push_back(c);
    }
    cut.push_back(size_);
    const size_t nchunk = cut.size() - 1;
    chunks_.assign(nchunk, Chunk());
    auto lex_chunk = [&](size_t k) {
        Chunk &ch = chunks_[k];
        const char *p = base_ + cut[k], *end = base_ + cut[k + 1];
        const bool last = k + 1 == nchunk;
        const size_t guess = (size_t)(end - p) / 10 + 2;
        ch.kind.reserve(guess);
        ch.a.reserve(guess);
        ch.b.reserve(guess);
        for (;;) {
            const char *nl = (const char *)std::memchr(p, '\n', (size_t)(end - p));
            const char *e = nl ? nl : end;
            if (!nl && !last) break;  // a non-final chunk ends with its '\n'
            uint32_t x = 0, y = 0;
            uint8_t kind;
            if (e == p) {
                kind = kEmpty;
            } else if (lex_data(p, e, &x, &y)) {
                kind = kData;
            } else {
                kind = kText;
                x = (uint32_t)ch.toff.size();
                y = (uint32_t)(e - p);
                ch.toff.push_back((uint64_t)(p - base_));
            }
            ch.kind.push_back(kind);
            ch.a.push_back(x);
            ch.b.push_back(y);
            if (!nl) break;
            p = nl + 1;
        }
    };
    std::vector<std::thread> pool;
    std::atomic<size_t> next{0};
    for (unsigned t = 0; t < std::min<size_t>(T, nchunk); ++t)
        pool.emplace_back([&] {
            for (size_t k; (k = next.fetch_add(1)) < nchunk;) lex_chunk(k);
        });
    for (auto &th : pool) th.join();
    if (size_ == 0) {  // an empty file reads as one empty line at end-of-file
        chunks_.assign(1, Chunk());
        chunks_[0].kind.push_back(kEmpty);
        chunks_[0].a.push_back(0);
        chunks_[0].b.push_back(0);
    }
    for (Chunk &ch : chunks_) {
        ch.first_line = lines_;
        lines_ += ch.kind.size();
    }
}

std::shared_ptr<const LexedFile> LexedFile::open(const std::string &fname) {
    static std::mutex mu;
    static std::unordered_map<std::string, std::weak_ptr<const LexedFile>> cache;
    std::lock_guard<std::mutex> lock(mu);
    if (auto sp = cache[fname].lock()) return sp;
    if (is_bz2(fname)) return nullptr;  // LineReader refuses it (gzio.cpp)
    if (is_gz(fname)) {
        std::shared_ptr<LexedFile> f(new LexedFile());
        if (!inflate_file(fname, f->inflated_)) return nullptr;
        f->size_ = f->inflated_.size();
        f->base_ = f->inflated_.data();
        f->lex_bytes();
        cache[fname] = f;
        return f;
    }
    const int fd = ::open(fname.c_str(), O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        ::close(fd);
        return nullptr;
    }
    std::shared_ptr<LexedFile> f(new LexedFile());
    f->lex(fname, fd, (uint64_t)st.st_size);
    ::close(fd);
    cache[fname] = f;
    return f;
}

// ---------------------------------------------------------------------------
// LineReader
// ---------------------------------------------------------------------------
LineReader::LineReader(const std::string &fname, bool lexed) {
    if (fname == "stdin") {
        fp_ = stdin;
        shown_ = "standard input stream";
    } else {
        const char *nl = std::getenv("UNIPEAK_NO_LEX");  // tests: the plain getline reader
        if (lexed && !(nl && *nl && *nl != '0')) lexed_ = LexedFile::open(fname);
        if (!lexed_) {
            fp_ = open_input(fname);  // ".gz" through zlib, ".bz2" refused (gzio.hpp)
            if (!fp_) {
                std::cerr << "error: could not read " << fname << std::endl << std::endl;
                exit_now(1);
            }
            owned_ = true;
        }
        shown_ = fname;
    }
    open_ = true;
}

LineReader::~LineReader() {
    close();
    std::free(buf_);
}

void LineReader::close() {
    if (open_ && owned_ && fp_) std::fclose(fp_);
    open_ = false;
    fp_ = nullptr;
}

const std::string &LineReader::read() {
    if (lexed_) {
        uint32_t p, c;
        if (next(&p, &c)) line_ = std::to_string(p) + " " + std::to_string(c);
        return line_;
    }
    ++line_no_;
    const ssize_t n = getline(&buf_, &cap_, fp_);
    if (n < 0) {
        eof_ = true;
        line_.clear();
        return line_;
    }
    size_t len = (size_t)n;
    if (len && buf_[len - 1] == '\n') --len;
    else eof_ = true;  // a last line without '\n' sets eofbit
    line_.assign(buf_, len);
    return line_;
}

bool LineReader::take_run(const LexedFile::Chunk **ch, size_t *b, size_t *e) {
    if (!lexed_ || !good()) return false;
    const auto &cs = lexed_->chunks();
    while (chunk_ < cs.size() && at_ >= cs[chunk_].kind.size()) {
        ++chunk_;
        at_ = 0;
    }
    if (chunk_ >= cs.size()) return false;
    const LexedFile::Chunk &c = cs[chunk_];
    size_t j = at_;
    while (j < c.kind.size() && c.kind[j] != LexedFile::kText) ++j;
    if (j == at_) return false;
    *ch = &c;
    *b = at_;
    *e = j;
    line_no_ += j - at_;
    at_ = j;
    if (line_no_ == lexed_->lines()) eof_ = true;
    return true;
}

bool LineReader::next(uint32_t *pos, uint32_t *count) {
    if (!lexed_) {
        read();
        return false;
    }
    ++line_no_;
    const auto &cs = lexed_->chunks();
    while (chunk_ < cs.size() && at_ >= cs[chunk_].kind.size()) {
        ++chunk_;
        at_ = 0;
    }
    if (chunk_ >= cs.size()) {  // past the end: what getline gives after eof
        eof_ = true;
        line_.clear();
        return false;
    }
    const LexedFile::Chunk &ch = cs[chunk_];
    const size_t i = at_++;
    if (line_no_ == lexed_->lines()) eof_ = true;
    switch (ch.kind[i]) {
    case LexedFile::kData:
        *pos = ch.a[i];
        *count = ch.b[i];
        return true;
    case LexedFile::kText:
        line_.assign(lexed_->bytes() + ch.toff[ch.a[i]], ch.b[i]);
        return false;
    default:
        line_.clear();
        return false;
    }
}

// ---------------------------------------------------------------------------
// ContigTable (regex ^(\w+)\W+(\d+), '#' comments, duplicate names fatal)
// ---------------------------------------------------------------------------
uint32_t ContigTable::index(const std::string &name) const {
    auto it = index_.find(name);
    return it == index_.end() ? size() : it->second;
}

void ContigTable::add(const std::string &name, uint32_t len) {
    if (index_.count(name)) fatal(name + " defined twice in contig table");
    index_[name] = (uint32_t)names_.size();
    names_.push_back(name);
    lens_.push_back(len);
    genome_ += len;
}

static bool word_char(int c) { return std::isalnum(c) || c == '_'; }

ContigTable ContigTable::parse(const std::string &fname) {
    std::cerr << "reading " << fname << "... " << std::flush;
    ContigTable t;
    LineReader in(fname);
    while (in.good()) {
        const std::string &l = in.read();
        if (l.empty() || l[0] == '#') continue;
        size_t i = 0;
        while (i < l.size() && word_char((unsigned char)l[i])) ++i;
        if (i == 0) continue;
        size_t j = i;
        while (j < l.size() && !word_char((unsigned char)l[j])) ++j;
        if (j == i) continue;
        size_t k = j;
        while (k < l.size() && std::isdigit((unsigned char)l[k])) ++k;
        if (k == j) continue;
        uint64_t v;
        if (!lex_uint(l.substr(j, k - j), 0xFFFFFFFFull, &v)) {
            std::cerr << "terminate called after throwing an instance of 'boost::bad_lexical_cast'" << std::endl;
            std::abort();
        }
        const std::string name = l.substr(0, i);
        if (t.index(name) != t.size()) {
            std::cerr << "error: " << name << " defined twice in contig table\n" << std::endl;
            exit_now(1);
        }
        t.add(name, (uint32_t)v);
    }
    if (t.size() == 0) {
        std::cerr << "error: no contigs in table" << std::endl << std::endl;
        exit_now(1);
    }
    std::cerr << t.size() << " contigs" << std::endl;
    return t;
}

// ---------------------------------------------------------------------------
// WigStream
// ---------------------------------------------------------------------------
WigStream::WigStream(const std::string &fname, const ContigTable *ct, int16_t offset,
                     uint16_t use_length, int strand_filter)
    : in_(fname, true), fname_(fname), ct_(ct), offset_(offset), use_length_(use_length),
      filter_(strand_filter) {
    name_ = fname_prefix(fname);
    a_.forward = true;
    a_.contig = 0;  // ParseAlignStream::open resets the contig to 0
}

void WigStream::bad(const char *what) const {
    if (t_defer_errors) throw DeferredError();
    std::cerr << "error: " << what << " in " << in_.display_name() << " line " << in_.line_no()
              << "\n" << std::endl;
    exit_now(1);
}

// name="(.+?)"
static bool name_quoted(const std::string &l, std::string *out) {
    for (size_t p = l.find("name=\""); p != std::string::npos; p = l.find("name=\"", p + 1)) {
        const size_t q = p + 6;
        if (q >= l.size()) continue;
        const size_t e = l.find('"', q + 1);
        if (e == std::string::npos) continue;
        *out = l.substr(q, e - q);
        return true;
    }
    return false;
}

// name=(.+?)<space>
static bool name_bare(const std::string &l, std::string *out) {
    for (size_t p = l.find("name="); p != std::string::npos; p = l.find("name=", p + 1)) {
        const size_t q = p + 5;
        if (q >= l.size()) continue;
        const size_t e = l.find(' ', q + 1);
        if (e == std::string::npos) continue;
        *out = l.substr(q, e - q);
        return true;
    }
    return false;
}

// "(.+) ([+-])" with a greedy first group
static bool strand_suffix(const std::string &name, std::string *expt, bool *fwd) {
    if (name.size() < 3) {
        if (name.size() < 3) return false;
    }
    for (size_t i = name.size() - 2; i >= 1; --i) {
        if (name[i] == ' ' && (name[i + 1] == '+' || name[i + 1] == '-')) {
            *expt = name.substr(0, i);
            *fwd = name[i + 1] == '+';
            return true;
        }
    }
    return false;
}

static bool starts(const std::string &l, const char *p) { return l.compare(0, std::strlen(p), p) == 0; }

void WigStream::parse(const std::string &l) {
    a_.count = 0;
    if (l.empty() || l[0] == '#') return;
    if (format_ == 0) {
        if (!starts(l, "track"))
            fatal("unsupported input format in " + fname_ + " (wiggle files only)");
        std::string nm;
        const bool has = name_quoted(l, &nm) || name_bare(l, &nm);
        if (has) name_ = nm;
        if (l.find("type=wiggle_0") == std::string::npos)
            fatal("unsupported input format in " + fname_ + " (wiggle files only)");
        std::string e;
        bool f;
        if (strand_suffix(name_, &e, &f)) {
            format_ = 6;
            name_ = e;
            a_.forward = f;
        } else {
            format_ = 7;
            name_ = has ? nm : std::string();
            a_.forward = true;
        }
        return;
    }
    if (std::isdigit((unsigned char)l[0])) {
        if (a_.contig == ct_->size()) return;
        const size_t d = l.find_last_of("\t ");
        if (d == std::string::npos) bad("bad format");
        uint64_t pos, cnt;
        if (!lex_uint(l.substr(0, d), 0xFFFFFFFFull, &pos)) bad("bad format");
        const size_t cs = d + (d + 1 < l.size() && l[d + 1] == '-' ? 2 : 1);
        if (!lex_uint(cs <= l.size() ? l.substr(cs) : std::string(), 0xFFFFFFFFull, &cnt)) bad("bad format");
        take((uint32_t)pos, (uint32_t)cnt);
        return;
    } else if (starts(l, "variableStep chrom=") && l.size() > 19) {
        a_.contig = ct_->index(l.substr(19));
        return;
    } else if (starts(l, "track")) {
        std::string nm;
        if (!name_quoted(l, &nm)) bad("bad format");
        a_.contig = ct_->size();
        name_ = nm;
        if (format_ == 6) {
            std::string e;
            bool f;
            if (!strand_suffix(name_, &e, &f)) bad("strand not defined");
            name_ = e;
            a_.forward = f;
        }
        return;
    } else {
        bad("bad format");
    }
}

// a data line's values under the stream's state (format.cpp:654-678): a.forward
// and a.contig hold the state; a.count ends 0 when the tag is out of bounds
static inline void place(uint32_t pos, uint32_t cnt, int format, uint16_t use_length, int16_t offset,
                         uint32_t size, Align &a, uint64_t &total, uint64_t &oob, uint64_t &confident) {
    a.first = pos;
    a.count = cnt;
    const uint32_t ext = use_length == 0 ? 0u : (uint32_t)(use_length - 1);
    if (format == 6) a.last = a.first + (a.forward ? ext : (uint32_t)(0u - ext));
    else a.last = a.first + ext;
    total += a.count;
    if (a.count == 0) return;
    if (use_length != 0) a.last = a.first + (a.forward ? ext : (uint32_t)(0u - ext));
    if (offset != 0) {
        if ((a.forward && (int)a.first > -offset) || (!a.forward && (int)a.last > offset)) {
            const uint32_t sh = (uint32_t)(a.forward ? (int)offset : -(int)offset);
            a.first += sh;
            a.last += sh;
        } else {
            oob += a.count;
            a.count = 0;
            return;
        }
    }
    if (a.first == 0 || a.first > size || a.last == 0 || a.last > size) {
        oob += a.count;
        a.count = 0;
        return;
    }
    confident += a.count;
}

void WigStream::take(uint32_t pos, uint32_t cnt) {
    place(pos, cnt, format_, use_length_, offset_, ct_->length(a_.contig), a_, total_, oob_, confident_);
}

bool WigStream::decode_rest(std::vector<Tag> &out, unsigned threads) {
    if (filter_ != 0 || !in_.lexed()) return false;
    // (A) serially: text lines through parse(), runs of other lines cut out
    // as segments with the state they start in
    struct Seg {
        const LexedFile::Chunk *ch = nullptr;
        size_t b = 0, e = 0;
        Align state;
        int format = 0;
        size_t at = 0;  // insertion point in out (records before it come first)
        std::vector<Tag> tags;
        uint64_t total = 0, oob = 0, confident = 0;
    };
    std::vector<Seg> segs;
    std::vector<std::pair<size_t, Tag>> texts;  // (segments before it, record)
    while (in_.good()) {
        const LexedFile::Chunk *ch;
        size_t b, e;
        if (in_.take_run(&ch, &b, &e)) {
            Seg g;
            g.ch = ch;
            g.b = b;
            g.e = e;
            g.state = a_;
            g.format = format_;
            segs.push_back(std::move(g));
            continue;
        }
        next_line();  // a text line (or end of file)
        if (a_.count != 0 && a_.contig != ct_->size())
            texts.push_back({segs.size(), Tag{a_.contig, a_.first, a_.count, a_.forward}});
    }
    // (B) the segments in parallel
    std::atomic<size_t> next{0};
    std::atomic<bool> unsupported{false};
    auto decode = [&] {
        for (size_t k; (k = next.fetch_add(1)) < segs.size();) {
            Seg &g = segs[k];
            Align a = g.state;
            if (a.contig == ct_->size()) continue;  // lines of unknown contigs are skipped
            const uint32_t size = ct_->length(a.contig);
            g.tags.reserve(g.e - g.b);
            for (size_t i = g.b; i < g.e; ++i) {
                if (g.ch->kind[i] != LexedFile::kData) continue;
                if (g.format == 0) {  // parse() would stop at this line
                    unsupported = true;
                    break;
                }
                place(g.ch->a[i], g.ch->b[i], g.format, use_length_, offset_, size, a, g.total, g.oob,
                      g.confident);
                if (a.count != 0) g.tags.push_back(Tag{a.contig, a.first, a.count, a.forward});
            }
        }
    };
    const unsigned T = (unsigned)std::min<size_t>(std::max(1u, threads), std::max<size_t>(1, segs.size()));
    auto run = [&](const std::function<void()> &fn) {
        next = 0;
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < T; ++t) pool.emplace_back(fn);
        fn();
        for (auto &th : pool) th.join();
    };
    run(decode);
    if (unsupported) fatal("unsupported input format in " + fname_ + " (wiggle files only)");
    // (C) place every record in line order: text records before the segment
    // that follows them, segments copied in parallel
    size_t n = out.size() + texts.size();
    std::vector<size_t> dest(segs.size());
    size_t ti = 0, w = out.size();
    for (size_t k = 0; k < segs.size(); ++k) {
        while (ti < texts.size() && texts[ti].first == k) ++ti, ++w;
        dest[k] = w;
        w += segs[k].tags.size();
        total_ += segs[k].total;
        oob_ += segs[k].oob;
        confident_ += segs[k].confident;
        n += segs[k].tags.size();
    }
    const size_t base = out.size();
    out.resize(n);
    w = base;
    ti = 0;
    for (size_t k = 0; k <= segs.size(); ++k) {
        while (ti < texts.size() && texts[ti].first == k) out[w++] = texts[ti++].second;
        if (k < segs.size()) w += segs[k].tags.size();
    }
    run([&] {
        for (size_t k; (k = next.fetch_add(1)) < segs.size();) {
            std::copy(segs[k].tags.begin(), segs[k].tags.end(), out.begin() + dest[k]);
            std::vector<Tag>().swap(segs[k].tags);
        }
    });
    a_.count = 0;
    a_.contig = ct_->size();
    return true;
}

// one line through the lexed fast path or the text parser; a lexed data
// line is what parse() would make of its text
void WigStream::next_line() {
    uint32_t pos, cnt;
    if (!in_.next(&pos, &cnt)) return parse(in_.line());
    a_.count = 0;
    if (format_ == 0) fatal("unsupported input format in " + fname_ + " (wiggle files only)");
    if (a_.contig == ct_->size()) return;
    take(pos, cnt);
}

void WigStream::read_plain() {
    if (in_.good()) {
        next_line();
    } else {
        a_.count = 0;
        a_.contig = ct_->size();
    }
    while ((a_.count == 0 || a_.contig == ct_->size()) && in_.good()) next_line();
}

const Align &WigStream::read_align() {
    read_plain();
    if (filter_ == 0) return a_;
    const bool want = filter_ == 1;
    if (format_ == 6 && want && !a_.forward && a_.count > 0) {  // forward handle is done
        a_.count = 0;
        in_.close();
    }
    while (in_.good() && a_.forward != want) read_plain();
    return a_;
}

uint64_t WigStream::expected_tags() {
    if (expected_ != 0) return expected_;
    while (in_.good()) {
        const std::string l = in_.read();
        if (!l.empty() && l[0] == '#') {
            const size_t m = l.find("# tags=");
            if (m != std::string::npos && m + 7 < l.size() && std::isdigit((unsigned char)l[m + 7])) {
                size_t k = m + 7;
                while (k < l.size() && std::isdigit((unsigned char)l[k])) ++k;
                uint64_t v;
                if (!lex_uint(l.substr(m + 7, k - m - 7), ~0ull, &v)) std::abort();
                if (expected_ == 0) expected_ = v;
                else bad("multiple tag count headers");
                if (expected_ == 0) bad("zero tag count");
            }
        } else {
            parse(l);
            if (expected_ == 0) {  // count the hard way
                WigStream t(fname_, ct_, offset_, use_length_, 0);
                while (t.in_.good()) t.read_plain();
                expected_ = t.confident_;
            }
            break;
        }
    }
    return expected_;
}

// ---------------------------------------------------------------------------
// SampleStream
// ---------------------------------------------------------------------------
SampleStream::SampleStream(const std::string &fname, const ContigTable *ct, int16_t offset,
                           uint16_t use_length, bool nondirectional)
    : fname_(fname), ct_(ct), offset_(offset), use_length_(use_length), nondir_(nondirectional) {
    if (!nondir_) {
        plain_.reset(new WigStream(fname, ct, offset, use_length, 0));
    } else {
        fwd_.reset(new WigStream(fname, ct, offset, use_length, 1));
        rev_.reset(new WigStream(fname, ct, offset, use_length, 2));
        // quirk Q18: the reference leaves this flag uninitialised; the
        // intended two-handle merge starts from the forward handle
        merged_.forward = true;
        merged_.contig = ct->size();
    }
}

std::unique_ptr<SampleStream> SampleStream::reopen() const {
    return std::unique_ptr<SampleStream>(new SampleStream(fname_, ct_, offset_, use_length_, nondir_));
}

uint64_t SampleStream::size_hint() const { return nondir_ ? fwd_->size_hint() : plain_->size_hint(); }

const WigStream &SampleStream::further() const {
    return fwd_->line_no() >= rev_->line_no() ? *fwd_ : *rev_;
}

uint64_t SampleStream::expected_tags() {
    if (!nondir_) return plain_->expected_tags();
    if (expected_ == 0)
        expected_ = fwd_->line_no() >= rev_->line_no() ? fwd_->expected_tags() : rev_->expected_tags();
    return expected_;
}

const std::string &SampleStream::expt_name() const { return nondir_ ? further().expt_name() : plain_->expt_name(); }
uint64_t SampleStream::confident() const { return nondir_ ? further().confident() : plain_->confident(); }
uint64_t SampleStream::out_of_bounds() const { return nondir_ ? further().out_of_bounds() : plain_->out_of_bounds(); }

// NondirParseAlignStream::readAlign (format.cpp:873-895)
const Align &SampleStream::read_align() {
    if (!nondir_) return plain_->read_align();
    if (merged_.forward) {
        const Align &f = fwd_->read_align();
        if (f.forward && f.contig == merged_.contig && f.first < merged_.first) {
            if (t_defer_errors) throw DeferredError();
            std::cerr << f.first << "\t" << merged_.first << "\n";
            fatal("alignments out of order");
        }
    } else {
        const Align &r = rev_->read_align();
        if (!r.forward && r.contig == merged_.contig && r.first < merged_.first)
            fatal("alignments out of order");
    }
    if (fwd_->line_no() == 0) fwd_->read_align();
    if (rev_->line_no() == 0) rev_->read_align();
    const Align &a1 = fwd_->last(), &a2 = rev_->last();
    bool lower;
    switch (2 * (a1.count == 0) + (a2.count == 0)) {
    case 0: lower = a1.contig == a2.contig ? a1.first <= a2.first : a1.contig < a2.contig; break;
    case 1: lower = true; break;
    case 2: lower = false; break;
    default: lower = true; break;
    }
    merged_ = lower ? a1 : a2;
    return merged_;
}

}  // namespace unipeak
