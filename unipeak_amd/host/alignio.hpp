// unipeak_amd/host/alignio.hpp -- the alignment side of bin/convert_align
// (SURVEY.md 8(f)4): ParseAlignStream's parser for every input format the
// reference reads (misc/format.cpp:69-86, 88-133, 213-232, 242-683, 693-705;
// BED, Eland multi, Corona, SAM, BAM, and the two wiggle formats), restated
// with the reference's counters, lexical_cast number rules, error messages
// and the state one parser carries from file to file (the established read
// length and its binomial posterior).  BAM goes through a BGZF reader on
// zlib (the reference vendors BamTools, misc/bamtools/, restated here only as
// far as convert_align reads it).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "wigio.hpp"

namespace unipeak {

// misc/data.hpp:37-43
struct Alignment {
    bool forward = true;
    uint32_t contig = 0;
    uint32_t first = 0, last = 0;
    std::string seq;
    uint32_t count = 0;
};

// misc/format.cpp:69-86
class BinomPosterior {
  public:
    explicit BinomPosterior(uint16_t read_length);
    double prob(uint16_t mismatches, const std::vector<uint32_t> &hits) const;

  private:
    std::vector<double> coef_;
};

class BamFile;  // BGZF-decompressed BAM records (alignio.cpp)

class AlignParser {
  public:
    AlignParser(const ContigTable *ct, uint16_t mismatch_tolerance, uint16_t use_length,
                int16_t offset, double prob_threshold);
    ~AlignParser();
    void open(const std::string &fname);
    void close();
    bool good() const;
    const Alignment &read_align();
    void print_summary() const;
    uint64_t total() const { return total_; }

  private:
    enum { kBed = 1, kElandMulti = 2, kCorona = 3, kSam = 4, kBam = 5, kDirWig = 6, kNondirWig = 7 };
    std::string read_line();
    void parse(const std::string &line);
    [[noreturn]] void error(const std::string &msg = "bad format") const;
    void parse_eland(const std::string &line);
    void parse_corona(const std::string &line);
    void parse_sam(const std::string &line);
    void parse_bam();
    void parse_wig(const std::string &line, bool directional);

    const ContigTable *ct_;
    const uint16_t tol_, use_len_;
    const int16_t offset_;
    uint16_t read_len_;
    const double prob_thr_, phred_thr_;
    std::unique_ptr<BinomPosterior> prob_;
    int format_ = 0;
    uint64_t total_ = 0, reject_ = 0, oob_ = 0, confident_ = 0;
    std::string name_, fname_;
    Alignment a_;
    std::unique_ptr<LineReader> in_;
    std::unique_ptr<BamFile> bam_;
    bool bam_done_ = false;
    uint64_t line_no_ = 0;  // InStream::lineNo_: never reset by open()
};

}  // namespace unipeak
