// unipeak_amd/host/gzio.cpp -- see gzio.hpp.  gzip streams are wrapped as
// stdio FILEs (fopencookie over zlib's gzFile), so every reader and writer of
// the CLIs keeps its FILE* code path.
#include "gzio.hpp"

#include <zlib.h>

#include <cerrno>
#include <cstring>

#include "wigio.hpp"

namespace unipeak {

static bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

bool is_gz(const std::string &fname) { return ends_with(fname, ".gz"); }
bool is_bz2(const std::string &fname) { return ends_with(fname, ".bz2"); }

[[noreturn]] static void no_bz2(const std::string &fname, const char *what) {
    fatal(std::string("could not ") + what + " " + fname +
          ": bzip2 (.bz2) streams are not supported by this build (libbz2 headers absent)");
}

[[noreturn]] static void gz_fail(gzFile g, const std::string &what) {
    int code = 0;
    const char *m = gzerror(g, &code);
    fatal(what + ": " + (m && *m ? m : "gzip stream error"));
}

namespace {
struct GzCookie {
    gzFile g;
    std::string name;
};

ssize_t gz_read(void *c, char *buf, size_t n) {
    GzCookie *k = (GzCookie *)c;
    const int r = gzread(k->g, buf, (unsigned)std::min<size_t>(n, 1u << 30));
    if (r < 0) gz_fail(k->g, "could not read " + k->name);
    return r;
}

ssize_t gz_write(void *c, const char *buf, size_t n) {
    GzCookie *k = (GzCookie *)c;
    size_t done = 0;
    while (done < n) {
        const int w = gzwrite(k->g, buf + done, (unsigned)std::min<size_t>(n - done, 1u << 30));
        if (w <= 0) return done ? (ssize_t)done : -1;
        done += (size_t)w;
    }
    return (ssize_t)done;
}

int gz_close(void *c) {
    GzCookie *k = (GzCookie *)c;
    const int r = gzclose(k->g);
    delete k;
    return r == Z_OK ? 0 : EOF;
}
// the reference's gzip filter (boost gzip_decompressor, misc/filterstream.cpp:
// 30-50) throws on a file without a gzip header; zlib would read it as plain
// bytes ("transparent" mode), so refuse it the same way
void not_gzip_check(gzFile g, const std::string &fname) {
    char c;
    const int r = gzread(g, &c, 1);  // reading decides direct vs gzip
    if (r < 0) gz_fail(g, "could not read " + fname);
    if (r == 1 && gzdirect(g)) {
        gzclose(g);
        fatal("could not read " + fname + ": not in gzip format");
    }
    if (r == 1) gzungetc((unsigned char)c, g);
}

// ISIZE of a gzip file (its last four bytes, little-endian), 0 if unreadable
size_t gz_isize_hint(const std::string &fname) {
    FILE *f = std::fopen(fname.c_str(), "rb");
    if (!f) return 0;
    unsigned char b[4] = {0, 0, 0, 0};
    size_t v = 0;
    if (std::fseek(f, -4, SEEK_END) == 0 && std::fread(b, 1, 4, f) == 4)
        v = (size_t)b[0] | ((size_t)b[1] << 8) | ((size_t)b[2] << 16) | ((size_t)b[3] << 24);
    std::fclose(f);
    return v;
}
}  // namespace

FILE *open_input(const std::string &fname) {
    if (is_bz2(fname)) no_bz2(fname, "read");
    if (!is_gz(fname)) return std::fopen(fname.c_str(), "rb");
    gzFile g = gzopen(fname.c_str(), "rb");
    if (!g) return nullptr;
    gzbuffer(g, 1u << 20);
    not_gzip_check(g, fname);
    cookie_io_functions_t io{gz_read, nullptr, nullptr, gz_close};
    GzCookie *k = new GzCookie{g, fname};
    FILE *f = fopencookie(k, "r", io);
    if (!f) {
        gzclose(g);
        delete k;
    }
    return f;
}

FILE *open_output(const std::string &fname) {
    if (is_bz2(fname)) no_bz2(fname, "write");
    if (!is_gz(fname)) return std::fopen(fname.c_str(), "wb");
    gzFile g = gzopen(fname.c_str(), "wb");
    if (!g) return nullptr;
    gzbuffer(g, 1u << 20);
    cookie_io_functions_t io{nullptr, gz_write, nullptr, gz_close};
    GzCookie *k = new GzCookie{g, fname};
    FILE *f = fopencookie(k, "w", io);
    if (!f) {
        gzclose(g);
        delete k;
    }
    return f;
}

bool inflate_file(const std::string &fname, std::string &out) {
    gzFile g = gzopen(fname.c_str(), "rb");
    if (!g) return false;
    gzbuffer(g, 1u << 20);
    not_gzip_check(g, fname);
    out.clear();
    // sized from the gzip trailer's ISIZE (the uncompressed length mod 2^32
    // of the last member): one allocation for files below 4 GiB instead of
    // doubling to up to twice the inflated size
    out.resize(gz_isize_hint(fname) + (1u << 16));
    size_t n = 0;
    for (;;) {
        if (out.size() - n < (1u << 16)) out.resize(out.size() + std::max<size_t>(out.size() / 4, 1u << 22));
        const int r = gzread(g, &out[n], (unsigned)std::min<size_t>(out.size() - n, 1u << 30));
        if (r < 0) gz_fail(g, "could not read " + fname);
        if (r == 0) break;
        n += (size_t)r;
    }
    out.resize(n);
    gzclose(g);
    return true;
}

}  // namespace unipeak
