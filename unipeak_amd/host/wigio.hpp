// unipeak_amd/host/wigio.hpp -- input side of the drop-in boundary:
// contig tables and the wiggle tag-frequency streams the reference's CLIs
// consume (misc/format.cpp:27-57, 242-272, 503-565, 654-705, 737-766,
// 798-811, 814-935; misc/data.cpp:196-261; misc/filterstream.cpp:66-72).
//
// Only the wiggle formats are accepted (alignment formats feed
// bin/convert_align, outside the path).  Everything is restated from the
// reference's behaviour: std::getline/istream::good() end-of-file
// semantics, boost::lexical_cast number rules, the contig-order driven
// stream consumption and the two-handle nondirectional merge.
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace unipeak {

[[noreturn]] void fatal(const std::string &msg);  // "error: ..." + exit(1)
[[noreturn]] void exit_now(int code);             // g_exit_hook, then std::exit
extern void (*g_exit_hook)();                     // e.g. join helper threads

// While set on a thread, input errors (fatal(), WigStream::bad()) throw
// DeferredError instead of printing and exiting: a read-ahead decode uses it
// to bail out to the serial replay, which then reports the error exactly
// where the reference would.
extern thread_local bool t_defer_errors;
struct DeferredError {};

// ---- misc/data.hpp:75-98 --------------------------------------------------
class ContigTable {
  public:
    uint32_t size() const { return (uint32_t)names_.size(); }
    uint32_t index(const std::string &name) const;  // size() if absent
    const std::string &name(uint32_t i) const { return names_[i]; }
    uint32_t length(uint32_t i) const { return i < lens_.size() ? lens_[i] : 0; }
    uint32_t genome_size() const { return genome_; }  // uint32: wraps (Q10)
    void add(const std::string &name, uint32_t len);
    static ContigTable parse(const std::string &fname);  // format.cpp:27-57

  private:
    std::vector<std::string> names_;
    std::vector<uint32_t> lens_;
    std::unordered_map<std::string, uint32_t> index_;
    uint32_t genome_ = 0;
};

// A file split into the lines std::getline would return -- count('\n') + 1
// of them, the last one (possibly empty) reaching end-of-file -- and lexed
// by a thread pool over newline-aligned chunks of the memory-mapped file
// (a ".gz" file is inflated into memory first, gzio.hpp).
// Lines of the canonical data form
// "<digits>< |\t>[-]<digits>" with both values < 2^32 are stored as two
// integers; every other line (track/variableStep headers, comments, anything
// unusual) keeps its text for the exact serial parser, so the lexed path
// changes speed only.  One instance per file name, shared by every handle
// that reads the file (both strand handles of a nondirectional sample and
// the counting pass of expected_tags).
class LexedFile {
  public:
    enum Kind : uint8_t { kEmpty = 0, kData = 1, kText = 2 };
    static std::shared_ptr<const LexedFile> open(const std::string &fname);  // null if unreadable
    ~LexedFile();
    uint64_t lines() const { return lines_; }
    struct Chunk {
        uint64_t first_line = 0;
        std::vector<uint8_t> kind;
        std::vector<uint32_t> a, b;  // data: pos, count; text: index into toff, length
        std::vector<uint64_t> toff;  // byte offsets of the text lines
    };
    const std::vector<Chunk> &chunks() const { return chunks_; }
    const char *bytes() const { return base_; }

  private:
    LexedFile() = default;
    void lex(const std::string &fname, int fd, uint64_t size);
    void lex_bytes();
    const char *base_ = nullptr;
    uint64_t size_ = 0, lines_ = 0;
    std::string inflated_;  // a ".gz" file's decompressed bytes (base_ points here)
    std::vector<Chunk> chunks_;
};

// host threads for ingest: UNIPEAK_THREADS, else min(16, hardware threads)
unsigned ingest_threads();

// std::getline + istream::good() semantics (filterstream.cpp:66-72); a
// regular file is read through its LexedFile, stdin line by line
class LineReader {
  public:
    explicit LineReader(const std::string &fname, bool lexed = false);
    ~LineReader();
    bool good() const { return open_ && !eof_; }
    const std::string &read();  // the next line without '\n'
    // lexed readers: the next line; true with *pos, *count set for a data
    // line, false with the text in line() otherwise
    bool next(uint32_t *pos, uint32_t *count);
    // lexed readers: the run of non-text lines at the cursor (within one
    // chunk) as [*b, *e) of *ch, consumed; false at a text line or the end
    bool take_run(const LexedFile::Chunk **ch, size_t *b, size_t *e);
    bool lexed() const { return (bool)lexed_; }
    const std::string &line() const { return line_; }
    void close();
    uint64_t line_no() const { return line_no_; }
    const std::string &display_name() const { return shown_; }
    uint64_t size_hint() const { return lexed_ ? lexed_->lines() : 0; }

  private:
    FILE *fp_ = nullptr;
    bool open_ = false, eof_ = false, owned_ = false;
    uint64_t line_no_ = 0;
    std::string line_, shown_;
    char *buf_ = nullptr;
    size_t cap_ = 0;
    std::shared_ptr<const LexedFile> lexed_;
    size_t chunk_ = 0, at_ = 0;
};

// one parsed alignment record (misc/data.hpp:27-43, wiggle subset)
struct Align {
    bool forward = true;
    uint32_t contig = 0;
    uint32_t first = 0, last = 0;
    uint32_t count = 0;
};

// a decoded record: what read_align() returns, minus the extent
struct Tag {
    uint32_t contig, first, count;
    bool forward;
};

// ParseAlignStream restricted to wiggle input; strand_filter 0: none,
// 1: forward only, 2: reverse only (StrandParseAlignStream)
class WigStream {
  public:
    WigStream(const std::string &fname, const ContigTable *ct, int16_t offset,
              uint16_t use_length, int strand_filter);
    const Align &read_align();  // next valid alignment (count 0 once exhausted)
    const Align &last() const { return a_; }
    uint64_t expected_tags();   // "# tags=N" header or a full counting pass
    const std::string &expt_name() const { return name_; }
    uint64_t confident() const { return confident_; }
    uint64_t out_of_bounds() const { return oob_; }
    uint64_t line_no() const { return in_.line_no(); }
    uint64_t size_hint() const { return in_.size_hint(); }
    // every further record read_align() would return, appended to out, the
    // stream left at end of input with the same counters; data lines are
    // decoded in parallel between header lines.  false (nothing read) for
    // strand-filtered handles and unlexed input.
    bool decode_rest(std::vector<Tag> &out, unsigned threads);

  private:
    void parse(const std::string &line);
    void take(uint32_t pos, uint32_t count);  // a data line's values (format.cpp:654-678)
    void next_line();
    void read_plain();
    [[noreturn]] void bad(const char *what) const;
    LineReader in_;
    std::string fname_;
    const ContigTable *ct_;
    int format_ = 0;  // 0 unknown, 6 directional wig, 7 nondirectional wig
    Align a_;
    std::string name_;
    uint64_t total_ = 0, oob_ = 0, confident_ = 0, expected_ = 0;
    int16_t offset_;
    uint16_t use_length_;
    int filter_;
};

// what a CLI reads one sample through: ParseAlignStream (directional) or
// NondirParseAlignStream (two handles merged by position, forward first)
class SampleStream {
  public:
    SampleStream(const std::string &fname, const ContigTable *ct, int16_t offset,
                 uint16_t use_length, bool nondirectional);
    SampleStream(SampleStream &&) = default;
    SampleStream &operator=(SampleStream &&) = default;
    // a second, independent stream over the same input (shares its lexed file)
    std::unique_ptr<SampleStream> reopen() const;
    uint64_t size_hint() const;  // lines in the input (0 if unknown)
    // WigStream::decode_rest for a directional stream; false otherwise
    bool decode_rest(std::vector<Tag> &out, unsigned threads) {
        return !nondir_ && plain_->decode_rest(out, threads);
    }
    const Align &read_align();
    const Align &last() const { return nondir_ ? merged_ : plain_->last(); }
    uint64_t expected_tags();
    const std::string &expt_name() const;
    uint64_t confident() const;
    uint64_t out_of_bounds() const;

  private:
    const WigStream &further() const;  // the handle that has read more lines
    std::string fname_;
    const ContigTable *ct_;
    int16_t offset_;
    uint16_t use_length_;
    bool nondir_;
    std::unique_ptr<WigStream> plain_, fwd_, rev_;
    Align merged_;
    uint64_t expected_ = 0;
};

// ---- number formats ---------------------------------------------------------
std::string fmt_lexical(double v);   // boost::lexical_cast<string>(double): %.17g
std::string fmt_ostream(double v);   // std::ostream << double, precision 6
std::string fmt_fixed2(double v);    // boost::format("%.2f")
bool lex_uint(const std::string &s, uint64_t maxv, uint64_t *out);  // lexical_cast<unsigned>
bool lex_short(const std::string &s, int16_t *out);
bool lex_double(const std::string &s, double *out);
std::vector<std::string> split_csv(const std::string &s);  // empty tokens dropped
std::string fname_prefix(const std::string &path);          // getFnamePrefix

}  // namespace unipeak
