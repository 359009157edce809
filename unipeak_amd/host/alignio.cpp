// unipeak_amd/host/alignio.cpp -- see alignio.hpp.
#include "alignio.hpp"

#include <zlib.h>

#include <cctype>
#include <cmath>
#include <cstring>
#include <iostream>
#include <regex>

namespace unipeak {

// ---------------------------------------------------------------------------
// BinomPosterior (misc/format.cpp:69-86)
// ---------------------------------------------------------------------------
BinomPosterior::BinomPosterior(uint16_t read_length) : coef_(read_length + 1) {
    const double c = 0.01 / (1 - 0.01);  // PROB_BASE_ERROR (misc/defaults.hpp:34)
    coef_[0] = 1;
    for (unsigned i = 1; i <= read_length; ++i) coef_[i] = coef_[i - 1] * c * (read_length - i + 1) / i;
}

double BinomPosterior::prob(uint16_t mismatches, const std::vector<uint32_t> &hits) const {
    if (!(mismatches < coef_.size() && hits.size() <= coef_.size())) {
        std::cerr << "convert_align: BinomPosterior::prob assertion failed" << std::endl;
        std::abort();  // the reference's assert (config.mk builds without NDEBUG)
    }
    const double numerator = coef_[mismatches];
    double denominator = 0;
    for (size_t i = 0; i < hits.size(); ++i) denominator += hits[i] * coef_[i];
    if (!(denominator > 0)) {
        std::cerr << "convert_align: BinomPosterior::prob assertion failed" << std::endl;
        std::abort();
    }
    return numerator / denominator;
}

// ---------------------------------------------------------------------------
// BAM through BGZF (what misc/bamtools/BamReader.cpp:561-700 reads): BGZF
// blocks are gzip members, inflated one after another into a sliding window
// that holds the current record (a few MB whatever the file size, as the
// reference's BamReader holds one block at a time)
// ---------------------------------------------------------------------------
class BamFile {
  public:
    ~BamFile();
    bool open(const std::string &fname);
    // next record; false at the end (or a truncated record)
    bool next();
    // fields of the current record (valid until the next call)
    int32_t ref_id = 0, pos = 0, l_seq = 0;
    uint16_t flag = 0;
    uint8_t mapq = 0;
    const uint8_t *tags = nullptr;
    uint32_t tag_len = 0;
    std::vector<std::string> ref_names;
    bool nm(uint32_t *out) const;  // BamAlignment::GetTag("NM", int32&)

  private:
    bool need(size_t n);  // n inflated bytes at at_; false if the stream ends first
    bool inflate_more();
    FILE *fp_ = nullptr;
    z_stream zs_;
    bool zinit_ = false, zdone_ = false, raw_eof_ = false;
    std::vector<uint8_t> raw_;
    size_t raw_at_ = 0;
    std::vector<uint8_t> data_;
    size_t at_ = 0;
};

static uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

BamFile::~BamFile() {
    if (zinit_) inflateEnd(&zs_);
    if (fp_) std::fclose(fp_);
}

// one inflate step of at most 1 MiB; false once nothing more will come (end
// of input, a truncated member or bytes that are not gzip: what inflated
// before stays readable, as the whole-file reader behaved)
bool BamFile::inflate_more() {
    if (zdone_) return false;
    if (raw_at_ == raw_.size() && !raw_eof_) {
        raw_.resize(1u << 20);
        const size_t k = std::fread(raw_.data(), 1, raw_.size(), fp_);
        raw_.resize(k);
        raw_at_ = 0;
        if (k == 0) raw_eof_ = true;
    }
    if (raw_at_ == raw_.size()) {  // input exhausted
        zdone_ = true;
        return false;
    }
    if (at_ > (8u << 20) && at_ * 2 > data_.size()) {  // slide the window
        data_.erase(data_.begin(), data_.begin() + (std::ptrdiff_t)at_);
        at_ = 0;
    }
    zs_.next_in = raw_.data() + raw_at_;
    zs_.avail_in = (uInt)(raw_.size() - raw_at_);
    const size_t old = data_.size(), room = 1u << 20;
    data_.resize(old + room);
    zs_.next_out = data_.data() + old;
    zs_.avail_out = (uInt)room;
    const int rc = inflate(&zs_, Z_NO_FLUSH);
    data_.resize(old + room - zs_.avail_out);
    raw_at_ = (size_t)(zs_.next_in - raw_.data());
    if (rc == Z_STREAM_END) {
        inflateReset(&zs_);  // the next BGZF block
    } else if (rc == Z_BUF_ERROR || (rc == Z_OK && zs_.avail_in == 0)) {
        if (raw_at_ == raw_.size() && raw_eof_) zdone_ = true;  // truncated member
    } else if (rc != Z_OK) {
        zdone_ = true;  // not gzip / corrupt
    }
    return true;
}

bool BamFile::need(size_t n) {
    while (data_.size() - at_ < n)
        if (!inflate_more() && data_.size() - at_ < n) return false;
    return true;
}

bool BamFile::open(const std::string &fname) {
    fp_ = std::fopen(fname.c_str(), "rb");
    if (!fp_) return false;
    std::memset(&zs_, 0, sizeof zs_);
    if (inflateInit2(&zs_, 15 + 16) != Z_OK) return false;
    zinit_ = true;
    // header: magic, text, references
    if (!need(12) || std::memcmp(data_.data() + at_, "BAM\1", 4) != 0) return false;
    at_ += 4;
    const uint32_t l_text = le32(&data_[at_]);
    if (!need(4 + (size_t)l_text + 4)) return false;
    at_ += 4 + l_text;
    const uint32_t n_ref = le32(&data_[at_]);
    at_ += 4;
    for (uint32_t i = 0; i < n_ref; ++i) {
        if (!need(4)) return false;
        const uint32_t l_name = le32(&data_[at_]);
        if (!need(4 + (size_t)l_name + 4)) return false;
        ref_names.emplace_back((const char *)&data_[at_ + 4], l_name ? l_name - 1 : 0);  // NUL-terminated
        at_ += 4 + l_name + 4;
    }
    return true;
}

bool BamFile::next() {
    if (!need(4)) return false;
    const uint32_t block = le32(&data_[at_]);
    if (block == 0 || block < 32 || !need(4 + (size_t)block)) return false;
    const uint8_t *r = &data_[at_ + 4];
    ref_id = (int32_t)le32(r);
    pos = (int32_t)le32(r + 4);
    const uint32_t bin_mq_nl = le32(r + 8), flag_nc = le32(r + 12);
    l_seq = (int32_t)le32(r + 16);
    mapq = (uint8_t)(bin_mq_nl >> 8);
    flag = (uint16_t)(flag_nc >> 16);
    const uint32_t l_name = bin_mq_nl & 0xff, n_cigar = flag_nc & 0xffff;
    const uint64_t core = 32ull + l_name + 4ull * n_cigar + (uint64_t)((l_seq + 1) / 2) + (uint64_t)l_seq;
    tags = core <= block ? r + core : r + block;
    tag_len = core <= block ? (uint32_t)(block - core) : 0;
    at_ += 4 + block;
    return true;
}

// BamAlignment::FindTag + GetTag(uint32&): misc/bamtools/BamAlignment.cpp:409-467
bool BamFile::nm(uint32_t *out) const {
    size_t p = 0;
    while (p + 3 <= tag_len) {
        const char t0 = (char)tags[p], t1 = (char)tags[p + 1], type = (char)tags[p + 2];
        p += 3;
        if (t0 == 'N' && t1 == 'M') {
            size_t len = 0;
            switch (type) {
            case 'A': case 'c': case 'C': len = 1; break;
            case 's': case 'S': len = 2; break;
            case 'i': case 'I': len = 4; break;
            case 'f': case 'Z': case 'H':
                std::fprintf(stderr, "ERROR: Cannot store tag of type %c in integer destination\n", type);
                return false;
            default:
                std::fprintf(stderr, "ERROR: Unknown tag storage class encountered: [%c]\n", type);
                return false;
            }
            uint32_t v = 0;
            for (size_t k = 0; k < len && p + k < tag_len; ++k) v |= (uint32_t)tags[p + k] << (8 * k);
            *out = v;
            return true;
        }
        // skip this tag's value
        switch (type) {
        case 'A': case 'c': case 'C': p += 1; break;
        case 's': case 'S': p += 2; break;
        case 'i': case 'I': case 'f': p += 4; break;
        case 'Z': case 'H':
            while (p < tag_len && tags[p]) ++p;
            ++p;
            break;
        case 'B': {
            if (p + 5 > tag_len) return false;
            const char sub = (char)tags[p];
            const uint32_t n = le32(&tags[p + 1]);
            const size_t w = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
            p += 5 + (size_t)n * w;
            break;
        }
        default: return false;
        }
    }
    return false;
}

// ---------------------------------------------------------------------------
// AlignParser
// ---------------------------------------------------------------------------
namespace {

bool starts_with(const std::string &s, const char *p) { return s.compare(0, std::strlen(p), p) == 0; }

// boost::split(fields, line, is_any_of(seps)): empty tokens kept
std::vector<std::string> split_any(const std::string &s, const char *seps) {
    std::vector<std::string> out;
    size_t b = 0;
    for (size_t i = 0; i <= s.size(); ++i)
        if (i == s.size() || (s[i] && std::strchr(seps, s[i]))) {
            out.push_back(s.substr(b, i - b));
            b = i + 1;
        }
    return out;
}

// boost::tokenizer<char_separator<char>>: empty tokens dropped
std::vector<std::string> tokens(const std::string &s, char sep) {
    std::vector<std::string> out;
    size_t b = 0;
    for (size_t i = 0; i <= s.size(); ++i)
        if (i == s.size() || s[i] == sep) {
            if (i > b) out.push_back(s.substr(b, i - b));
            b = i + 1;
        }
    return out;
}

// misc/format.hpp:24-33 (format detection runs once per file)
const std::regex &bed_re() { static const std::regex r("^[^\\s]+\\s\\d+\\s\\d+\\s[^\\s]*\\s[^\\s]*?\\s[+-]"); return r; }
const std::regex &eland_re() { static const std::regex r("^>.+?\\t[ACGTN\\.]+\\t(\\d+:\\d+:\\d+|RM|NM|QC)\\t.+"); return r; }
const std::regex &corona_re() { static const std::regex r("^>\\d+_\\d+_\\d+_F3"); return r; }
const std::regex &sam_header_re() { static const std::regex r("^@[A-Za-z][A-Za-z](\\t[A-Za-z][A-Za-z0-9]:[ -~]+)+$"); return r; }

// NAME_REGEX1 name="(.+?)"
bool name_quoted(const std::string &l, std::string *out) {
    for (size_t k = l.find("name=\""); k != std::string::npos; k = l.find("name=\"", k + 1)) {
        const size_t e = l.find('"', k + 7);  // (.+?): at least one character
        if (e != std::string::npos) {
            *out = l.substr(k + 6, e - k - 6);
            return true;
        }
    }
    return false;
}
// NAME_REGEX2 name=(.+?) (a space ends it)
bool name_plain(const std::string &l, std::string *out) {
    for (size_t k = l.find("name="); k != std::string::npos; k = l.find("name=", k + 1)) {
        const size_t e = l.find(' ', k + 6);
        if (e != std::string::npos) {
            *out = l.substr(k + 5, e - k - 5);
            return true;
        }
    }
    return false;
}
// DIRECTIONAL_WIG_NAME_REGEX (.+) ([+-]): the last " +"/" -" after one character
bool dir_name(const std::string &n, std::string *name, bool *fwd) {
    for (size_t k = n.size() >= 2 ? n.size() - 2 : 0; k >= 1 && k + 1 < n.size(); --k)
        if (n[k] == ' ' && (n[k + 1] == '+' || n[k + 1] == '-')) {
            *name = n.substr(0, k);
            *fwd = n[k + 1] == '+';
            return true;
        }
    return false;
}

bool lex_u32(const std::string &s, uint32_t *v) {
    uint64_t x;
    if (!lex_uint(s, 0xFFFFFFFFull, &x)) return false;
    *v = (uint32_t)x;
    return true;
}
bool lex_u16(const std::string &s, uint16_t *v) {
    uint64_t x;
    if (!lex_uint(s, 0xFFFFull, &x)) return false;
    *v = (uint16_t)x;
    return true;
}

struct BadCast {};
uint32_t u32_or_throw(const std::string &s) {
    uint32_t v;
    if (!lex_u32(s, &v)) throw BadCast();
    return v;
}
uint16_t u16_or_throw(const std::string &s) {
    uint16_t v;
    if (!lex_u16(s, &v)) throw BadCast();
    return v;
}

}  // namespace

AlignParser::AlignParser(const ContigTable *ct, uint16_t tol, uint16_t use_len, int16_t offset, double prob_thr)
    : ct_(ct), tol_(tol), use_len_(use_len), offset_(offset), read_len_(use_len), prob_thr_(prob_thr),
      phred_thr_(prob_thr == 0 ? 0 : prob_thr == 1 ? 255 : -10 * std::log10(1 - prob_thr)),
      prob_(use_len == 0 ? nullptr : new BinomPosterior(use_len)) {}

AlignParser::~AlignParser() = default;

void AlignParser::close() {
    bam_.reset();
    in_.reset();
}

// ParseAlignStream::open (misc/format.cpp:103-128); the line counter of the
// underlying InStream is not reset between files
void AlignParser::open(const std::string &fname) {
    close();
    if (fname.size() >= 4 && fname.compare(fname.size() - 4, 4, ".bam") == 0) {
        bam_.reset(new BamFile);
        if (!bam_->open(fname)) bam_done_ = true;  // BamReader::Open failed: IsOpen() false
        else bam_done_ = false;
        format_ = kBam;
        fname_ = fname;
    } else {
        in_.reset(new LineReader(fname));
        format_ = 0;
        fname_ = in_->display_name();
    }
    total_ = reject_ = oob_ = confident_ = 0;
    name_ = fname_prefix(fname);
    a_ = Alignment();
}

bool AlignParser::good() const {
    if (format_ == kBam) return bam_ && !bam_done_;
    return in_ && in_->good();
}

std::string AlignParser::read_line() {
    if (format_ == kBam) return "";
    ++line_no_;
    return in_->read();
}

void AlignParser::error(const std::string &msg) const {
    std::cerr << "error: " << msg << " in " << fname_ << " line " << line_no_ << "\n" << std::endl;
    exit_now(1);
}

// ParseAlignStream::readAlign (misc/format.cpp:693-705)
const Alignment &AlignParser::read_align() {
    if (good()) {
        parse(read_line());
    } else {
        a_.count = 0;
        a_.contig = ct_->size();
    }
    while ((a_.count == 0 || a_.contig == ct_->size()) && good()) parse(read_line());
    return a_;
}

void AlignParser::print_summary() const {
    if (!name_.empty()) std::cerr << name_ << ": ";
    std::cerr << total_ << " tags";
    if (format_ == kElandMulti || format_ == kCorona || format_ == kSam || format_ == kBam) {
        char pct[64];
        std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)confident_ / (double)total_);
        std::cerr << "\n  " << confident_ << (prob_thr_ != 0 ? " confidently mapped" : " unique best")
                  << " hits (" << pct << "%)";
        if (prob_thr_ != 0) {
            std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)reject_ / (double)total_);
            std::cerr << "\n  " << reject_ << " unique best hits rejected by filter (" << pct << "%)";
        }
    }
    if (oob_ > 0) std::cerr << "\n" << oob_ << " out of contig bounds";
    std::cerr << std::endl;
}

// ParseAlignStream::parseAlign (misc/format.cpp:242-683)
void AlignParser::parse(const std::string &line) {
    a_.count = 0;
    try {
        if ((line.empty() && format_ != kBam) || (!line.empty() && line[0] == '#')) return;
        if (format_ == 0) {
            if (starts_with(line, "track")) {
                std::string n;
                const bool named = name_quoted(line, &n) || name_plain(line, &n);
                if (named) name_ = n;
                if (line.find("type=wiggle_0") != std::string::npos) {
                    std::string dn;
                    bool f;
                    if (dir_name(name_, &dn, &f)) {
                        format_ = kDirWig;
                        name_ = dn;
                        a_.forward = f;
                    } else {
                        format_ = kNondirWig;
                        name_ = named ? n : std::string();  // matches[1] of a failed search
                        a_.forward = true;
                    }
                } else {
                    format_ = kBed;
                }
                return;
            } else if (std::regex_search(line, bed_re())) {
                format_ = kBed;
            } else if (std::regex_search(line, eland_re())) {
                format_ = kElandMulti;
            } else if (std::regex_search(line, corona_re())) {
                format_ = kCorona;
            } else if (std::regex_search(line, sam_header_re())) {
                format_ = kSam;
            } else {
                error();
            }
        }
        switch (format_) {
        case kBed: {
            if (starts_with(line, "track")) break;
            const std::vector<std::string> f = split_any(line, "\t ");
            if (f.size() < 6) error();
            const char strand = f[5].empty() ? '\0' : f[5][0];
            if (strand == '+') a_.forward = true;
            else if (strand == '-') a_.forward = false;
            else error();
            a_.contig = ct_->index(f[0]);
            a_.seq = f[3];
            if (a_.forward) {
                a_.first = u32_or_throw(f[1]) + 1;
                a_.last = u32_or_throw(f[2]);
            } else {
                a_.first = u32_or_throw(f[2]);
                a_.last = u32_or_throw(f[1]) + 1;
            }
            a_.count = 1;
            ++total_;
            break;
        }
        case kElandMulti: parse_eland(line); break;
        case kCorona: parse_corona(line); break;
        case kDirWig: parse_wig(line, true); if (a_.count == 0) return; break;
        case kNondirWig: parse_wig(line, false); if (a_.count == 0) return; break;
        case kSam: parse_sam(line); break;
        case kBam: parse_bam(); break;
        }
        if (a_.count != 0 && a_.contig != ct_->size()) {
            if (read_len_ != 0) a_.last = a_.first + (a_.forward ? read_len_ - 1 : -(read_len_ - 1));
            if (offset_ != 0) {  // avoid shifting off the left end
                if ((a_.forward && ((int)a_.first > -offset_)) || (!a_.forward && ((int)a_.last > offset_))) {
                    a_.first += (a_.forward ? offset_ : -offset_);
                    a_.last += (a_.forward ? offset_ : -offset_);
                } else {
                    oob_ += a_.count;
                    a_.count = 0;
                    return;
                }
            }
            const uint32_t size = ct_->length(a_.contig);
            if (a_.first == 0 || a_.first > size || a_.last == 0 || a_.last > size) {
                oob_ += a_.count;
                a_.count = 0;
                return;
            }
            confident_ += a_.count;
        }
    } catch (const BadCast &) {
        error();
    }
}

// misc/format.cpp:314-429
void AlignParser::parse_eland(const std::string &line) {
    const std::vector<std::string> f = split_any(line, "\t");
    if (f.size() < 4) error();
    ++total_;
    if (f[3] == "-") return;
    std::vector<uint32_t> counts;
    uint16_t best_mm = 0;
    bool found_best = false, unique = false;
    for (const std::string &t : tokens(f[2], ':')) {
        counts.push_back(u32_or_throw(t));
        if (!found_best) {
            if (best_mm > tol_) break;  // the unique best fails the mismatch tolerance
            if (counts.back() == 0) {
                ++best_mm;
            } else {
                found_best = true;
                if (counts.back() == 1) unique = true;
                else break;
            }
        }
    }
    if (!unique) return;
    a_.seq = f[1];
    std::string use_seq = a_.seq;
    if (use_len_ != 0) {
        if (a_.seq.size() >= use_len_) use_seq = a_.seq.substr(0, use_len_);
        else error("sequence shorter than requested length");
    } else if (read_len_ != 0) {
        if (use_seq.size() != read_len_) error("different read length");
    } else {
        read_len_ = (uint16_t)a_.seq.size();
        if (prob_thr_ != 0) prob_.reset(new BinomPosterior(read_len_));
    }
    uint16_t nN = 0;
    for (char ch : use_seq) nN += ch == 'N';
    if (prob_ && prob_->prob(best_mm, counts) < prob_thr_) {
        a_.count = 0;
        ++reject_;
        return;
    }
    for (std::string hit : tokens(f[3], ',')) {
        const size_t colon = hit.find(':');
        if (colon != std::string::npos) {
            const std::string cs = hit.substr(0, colon);
            const size_t slash = cs.find('/');
            a_.contig = ct_->index(fname_prefix(slash == std::string::npos ? cs : cs.substr(slash + 1)));
            hit.erase(0, colon + 1);
        }
        const size_t dir = hit.find_first_of("FR");
        if (dir == std::string::npos) error();
        const uint32_t left = u32_or_throw(hit.substr(0, dir));
        a_.forward = hit[dir] == 'F';
        hit.erase(0, dir + 1);
        uint16_t mm = 0, elapsed = 0;
        size_t w = hit.find_first_of("ACGTN");
        if (w == std::string::npos) {
            const uint16_t v = u16_or_throw(hit);
            if (v <= 2) mm = v;  // Eland reports only the number of mismatches
        } else {
            while (w != std::string::npos) {
                if (w > 0) elapsed += u16_or_throw(hit.substr(0, w));
                if (elapsed >= use_seq.size()) break;
                if (hit[w] != 'N') ++mm;
                ++elapsed;
                hit.erase(0, w + 1);
                w = hit.find_first_of("ACGTN");
            }
            mm -= nN;  // Eland doesn't count Ns as mismatches, but reports them
        }
        if (mm == best_mm) {
            a_.first = left + (a_.forward ? 0 : read_len_ - 1);
            if (a_.contig < ct_->size()) a_.count = 1;
            break;
        }
    }
}

// misc/format.cpp:431-501
void AlignParser::parse_corona(const std::string &line) {
    if (!starts_with(line, ">")) return;
    a_.seq = read_line();
    ++total_;
    const size_t at = line.find(',');
    if (at == std::string::npos) return;
    if (use_len_ == 0) {
        if (read_len_ != 0) {
            if (a_.seq.size() - 1 != read_len_) error("different read length");
        } else {
            read_len_ = (uint16_t)(a_.seq.size() - 1);
            if (prob_thr_ != 0) prob_.reset(new BinomPosterior(read_len_));
        }
    } else if (a_.seq.size() - 1 < use_len_) {
        error("sequence shorter than requested length");
    }
    uint16_t best_mm = (uint16_t)(tol_ + 1);
    std::vector<uint32_t> mmc(1, 0);
    for (const std::string &h : split_any(line.substr(at + 1), ",")) {
        const std::vector<std::string> f = split_any(h, ".");
        if (f.size() != 3) error();
        const uint32_t contig = ct_->index(f[0]);
        if (contig >= ct_->size()) break;
        const uint16_t mm = u16_or_throw(f[2]);
        if (prob_thr_ != 0) {
            if (mmc.size() >= (uint16_t)(mm + 1)) {
                ++mmc[mm];
            } else {
                while (mmc.size() < mm) mmc.push_back(0);
                mmc.push_back(1);
            }
        }
        if (mm < best_mm) {
            a_.contig = contig;
            if (!starts_with(f[1], "-")) {
                a_.forward = true;
                a_.first = u32_or_throw(f[1]) + 1;
            } else {
                a_.forward = false;
                a_.first = u32_or_throw(f[1].substr(1)) + 1;
            }
            best_mm = mm;
            a_.count = 1;
        } else if (mm == best_mm) {
            a_.count = 0;
            if (best_mm == 0) break;  // non-unique
        }
    }
    if (prob_ && a_.count != 0 && prob_->prob(best_mm, mmc) < prob_thr_) {
        a_.count = 0;
        ++reject_;
    }
}

// misc/format.cpp:503-565 (both wiggle formats)
void AlignParser::parse_wig(const std::string &line, bool directional) {
    if (!line.empty() && std::isdigit((unsigned char)line[0])) {
        if (a_.contig == ct_->size()) return;  // contig not defined or not in the table
        const size_t d = line.find_last_of("\t ");
        if (d == std::string::npos) error();
        a_.first = u32_or_throw(line.substr(0, d));
        a_.count = u32_or_throw(line.substr(d + (d + 1 < line.size() && line[d + 1] == '-' ? 2 : 1)));
        if (directional)
            a_.last = a_.first + (use_len_ == 0 ? 0 : (a_.forward ? use_len_ - 1 : -(use_len_ - 1)));
        else
            a_.last = a_.first + (use_len_ == 0 ? 0 : use_len_ - 1);
        total_ += a_.count;
    } else if (starts_with(line, "variableStep chrom=") && line.size() > 19) {
        a_.contig = ct_->index(line.substr(19));
    } else if (starts_with(line, "track") && name_quoted(line, &name_)) {
        a_.contig = ct_->size();
        if (directional) {
            std::string dn;
            bool f;
            if (!dir_name(name_, &dn, &f)) error("strand not defined");
            name_ = dn;
            a_.forward = f;
        }
    } else {
        error();
    }
}

// misc/format.cpp:567-610
void AlignParser::parse_sam(const std::string &line) {
    if (!line.empty() && line[0] == '@') return;
    const std::vector<std::string> f = split_any(line, "\t");
    if (f.size() < 10) error();
    const uint16_t flag = u16_or_throw(f[1]);
    if (flag & 0x0100) return;  // non-primary
    ++total_;
    if (flag & (0x0004 + 0x0200)) return;  // unmapped or failed QC
    if (f.size() > 11) {
        int64_t ed = 0;
        for (const std::string &x : f)  // SAM_EDITDISTANCE_REGEX ^NM:i:(\d+)$ over every field
            if (x.size() > 5 && starts_with(x, "NM:i:") &&
                x.find_first_not_of("0123456789", 5) == std::string::npos) {
                uint64_t v;
                if (!lex_uint(x.substr(5), 0x7FFFFFFFull, &v)) throw BadCast();
                ed = (int64_t)v;
                break;
            }
        if (ed > tol_) return;
    }
    if (phred_thr_ != 0 && phred_thr_ != 255 && u16_or_throw(f[4]) < phred_thr_) {
        ++reject_;
        return;
    }
    a_.contig = ct_->index(f[2]);
    if (a_.contig == ct_->size()) return;
    a_.seq = f[9];
    if (use_len_ != 0 && a_.seq.size() < use_len_) error("sequence shorter than requested length");
    a_.forward = !(flag & 0x0010);
    a_.first = u32_or_throw(f[3]) + (a_.forward ? 0 : (uint32_t)a_.seq.size() - 1);
    a_.last = a_.first + (a_.forward ? 1 : -1) * (int)((use_len_ != 0 ? use_len_ : a_.seq.size()) - 1);
    a_.count = 1;
}

// misc/format.cpp:612-647
void AlignParser::parse_bam() {
    if (!bam_ || !bam_->next()) {
        bam_done_ = true;
        return;
    }
    const uint16_t flag = bam_->flag;
    if (flag & 0x0100) return;  // !IsPrimaryAlignment
    ++total_;
    if ((flag & 0x0200) || (flag & 0x0004)) return;  // IsFailedQC || !IsMapped
    uint32_t nm;
    if (bam_->nm(&nm) && (int32_t)nm > tol_) return;
    if (phred_thr_ != 0 && phred_thr_ != 255 && bam_->mapq < phred_thr_) {
        ++reject_;
        return;
    }
    const int32_t rid = bam_->ref_id;
    const std::string name = (rid >= 0 && (size_t)rid < bam_->ref_names.size()) ? bam_->ref_names[rid] : "";
    a_.contig = ct_->index(name);
    if (a_.contig == ct_->size()) return;
    a_.seq.clear();  // only its length matters below (Length = l_seq)
    a_.forward = !(flag & 0x0010);
    const int32_t len = bam_->l_seq;
    a_.first = (uint32_t)bam_->pos + (a_.forward ? 1 : (uint32_t)len);
    a_.last = a_.first + (a_.forward ? 1 : -1) * (int)((use_len_ != 0 ? use_len_ : len) - 1);
    a_.count = 1;
}

}  // namespace unipeak
