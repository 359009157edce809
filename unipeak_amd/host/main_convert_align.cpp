// bin/convert_align -- drop-in for src/convert_align.cpp (SURVEY.md 3.5,
// 8(f)4): alignment files -> a wiggle tag-frequency file, the input the path
// reads.  Parsing is the reference's ParseAlignStream (alignio.cpp, one
// parser carried across the files); the CountMap -- per (strand, contig)
// position -> count -- lives on the GPU as dense HBM tracks (countmap.hip),
// and its ordered walk is a device stream compaction.  The wiggle writer is
// FormatOutStream's (misc/format.cpp:1003-1089, 1164-1219).
#include <algorithm>
#include <cstdio>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "alignio.hpp"
#include "cli.hpp"
#include "unipeak_hip.h"
#include "wigio.hpp"
#include "gzio.hpp"

using namespace unipeak;

namespace {

// one batch of parsed alignments on its way to the device
struct Batch {
    std::vector<uint32_t> contig, pos, count;
    std::vector<uint8_t> fwd;
    bool unit = true;  // every count is 1 (alignment formats): no count upload
    size_t size() const { return pos.size(); }
    void clear() {
        contig.clear();
        pos.clear();
        count.clear();
        fwd.clear();
        unit = true;
    }
};

std::thread g_warm;
void join_warm() {
    if (g_warm.joinable()) g_warm.join();
}

std::string track_header(const std::string &name, bool directional, bool fwd, const std::string &assembly) {
    std::string s = "track name=\"" + name;
    if (directional) s += fwd ? " +" : " -";
    s += "\"";
    if (directional) s += std::string(" description=\"") + (fwd ? name : " ") + "\"";
    s += " priority=3 visibility=full type=wiggle_0 alwaysZero=on color=";  // ALIGN_PRIORITY
    if (!directional) s += "191,0,191";
    else s += fwd ? "0,0,255" : "255,0,0 altColor=255,0,0";
    if (!assembly.empty()) s += " db=" + assembly;
    return s + "\n";
}

}  // namespace

int main(int argc, char **argv) {
    ArgParser ap({{"q", "quiet", true, false},     {"D", "non-directional", true, false},
                  {"i", "mismatches", false, false}, {"l", "length", false, false},
                  {"s", "shift", false, false},      {"p", "prob", false, false},
                  {"a", "assembly", false, false},   {"n", "name", false, false},
                  {"c", "contigs", false, true},     {"o", "output", false, true}});
    ap.parse(argc, argv);
    const std::vector<std::string> files = ap.files();
    if (files.empty()) {
        std::cerr << "error: Required argument missing for arg align filenames\n" << std::endl;
        return 1;
    }
    const bool quiet = ap.on("q"), directional = !ap.on("D");
    const uint16_t tol = (uint16_t)ap.uint("i", 1, 0xFFFF);  // DEFAULT_MISMATCH_TOLERANCE
    const uint16_t use_len = (uint16_t)ap.uint("l", 0, 0xFFFF);
    int16_t offset = 0;
    if (ap.on("s") && !lex_short(ap.str("s"), &offset)) {
        std::cerr << "error: Couldn't read argument value from string '" << ap.str("s")
                  << "' for arg -s (--shift)\n" << std::endl;
        return 1;
    }
    const double prob = ap.dbl("p", 0.9);  // DEFAULT_PROB_THRESHOLD
    const std::string assembly = ap.str("a");
    std::string track = ap.str("n");
    const std::string out_name = ap.str("o"), ct_name = ap.str("c");
    const ContigTable ct = ContigTable::parse(ct_name);
    PhaseTimer timer;

    // the device (and its dense tracks) comes up while the first file parses
    up_cm *cm = nullptr;
    int cm_err = UP_OK;
    g_warm = std::thread([&] {
        int nd = 0;
        up_device_count(&nd);
        if (nd < 1) {
            cm_err = UP_E_NODEV;
            return;
        }
        std::vector<uint32_t> lens(ct.size());
        for (uint32_t c = 0; c < ct.size(); ++c) lens[c] = ct.length(c);
        cm_err = up_cm_open(0, ct.size(), lens.data(), &cm);
    });
    auto device = [&]() -> up_cm * {
        join_warm();
        if (cm_err == UP_E_NODEV) fatal("no HIP device available (the GPU path has no CPU fallback)");
        if (cm_err != UP_OK) fatal(std::string("convert_align on the GPU failed: ") + up_strerror(cm_err));
        return cm;
    };
    g_exit_hook = join_warm;  // an input error must not exit mid-initialisation

    uint64_t tag_count = 0;  // CountMap::tagCount
    Batch b;
    const size_t kBatch = 1u << 24;
    auto flush = [&] {
        if (!b.size()) return;
        const int e = up_cm_add(device(), b.size(), b.contig.data(), b.pos.data(), b.fwd.data(),
                                b.unit ? nullptr : b.count.data());
        if (e != UP_OK) fatal(std::string("convert_align on the GPU failed: ") + up_strerror(e));
        b.clear();
    };
    AlignParser in(&ct, tol, use_len, offset, prob);
    for (const std::string &f : files) {
        in.open(f);
        std::cerr << "reading " << f << "..." << std::endl;
        if (!quiet) std::cerr << "0 tags read";
        while (in.good()) {
            const Alignment &a = in.read_align();
            if (a.count && a.contig < ct.size()) {  // CountMap::add (misc/data.cpp:301-314)
                b.contig.push_back(a.contig);
                b.pos.push_back(a.first);
                b.fwd.push_back(a.forward ? 1 : 0);
                b.count.push_back(a.count);
                b.unit = b.unit && a.count == 1;
                tag_count += a.count;
                if (b.size() >= kBatch) flush();
            }
        }
        in.close();
        if (!quiet) std::cerr << "\r";
        in.print_summary();
    }
    timer.mark("parse");
    std::cerr << tag_count << " usable tags" << std::endl;
    if (tag_count == 0) {
        join_warm();
        std::cerr << "error: nothing to do\n" << std::endl;
        return 1;
    }
    flush();
    if (track.empty()) track = fname_prefix(out_name);
    std::cerr << "writing " << out_name << " in wiggle format with "
              << (directional ? "separate strands" : "strands combined") << "... " << std::flush;

    // the CountMap's iterator order, compacted on the device
    up_cm *h = device();
    uint64_t n = 0;
    int e = up_cm_collect(h, directional ? 0 : 1, &n, nullptr, nullptr, nullptr, nullptr, 0);
    std::vector<uint32_t> oc(n), op(n), on(n);
    std::vector<uint8_t> of(n);
    if (e == UP_OK) e = up_cm_collect(h, directional ? 0 : 1, &n, oc.data(), op.data(), on.data(), of.data(), n);
    if (e != UP_OK) fatal(std::string("convert_align on the GPU failed: ") + up_strerror(e));
    up_cm_close(h);
    timer.mark("gpu");

    std::string head;
    for (const std::string &f : files) head += "# original_file=" + f + "\n";
    if (prob != 0) head += "# prob_threshold=" + fmt_lexical(prob) + "\n";
    head += "# tags=" + std::to_string(tag_count) + "\n";
    // format the entries in parallel chunks (a track header where the
    // strand or -- nondirectional -- the first entry changes, a
    // variableStep line where the contig changes)
    const unsigned T = std::max(1u, std::min<unsigned>(ingest_threads(), (unsigned)(n / 65536 + 1)));
    std::vector<std::string> part(T);
    std::vector<uint64_t> written(T, 0);
    {
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < T; ++t)
            pool.emplace_back([&, t] {
                const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
                std::string &s = part[t];
                s.reserve((hi - lo) * 14);
                char buf[40];
                for (uint64_t i = lo; i < hi; ++i) {
                    const bool first = i == 0;
                    if (directional) {
                        if (first || of[i] != of[i - 1]) s += track_header(track, true, of[i], assembly);
                        if (first || of[i] != of[i - 1] || oc[i] != oc[i - 1])
                            s += "variableStep chrom=" + ct.name(oc[i]) + "\n";
                        const int k = std::snprintf(buf, sizeof buf, of[i] ? "%u %u\n" : "%u -%u\n", op[i], on[i]);
                        s.append(buf, (size_t)k);
                    } else {
                        if (first) s += track_header(track, false, true, assembly);
                        if (first || oc[i] != oc[i - 1]) s += "variableStep chrom=" + ct.name(oc[i]) + "\n";
                        const int k = std::snprintf(buf, sizeof buf, "%u %u\n", op[i], on[i]);
                        s.append(buf, (size_t)k);
                    }
                    written[t] += on[i];
                }
            });
        for (auto &th : pool) th.join();
    }
    FILE *out = out_name == "stdout" ? stdout : open_output(out_name);
    if (!out) {
        std::cerr << "error: could not write " << out_name << std::endl << std::endl;
        return 1;
    }
    std::fwrite(head.data(), 1, head.size(), out);
    uint64_t out_tags = 0;
    for (unsigned t = 0; t < T; ++t) {
        std::fwrite(part[t].data(), 1, part[t].size(), out);
        out_tags += written[t];
    }
    if (out != stdout) std::fclose(out);
    else std::fflush(stdout);
    timer.mark("write");
    if (out_tags != tag_count) {  // the reference's self-check (src/convert_align.cpp:137-140)
        std::cerr << "error: " << out_tags << " " << tag_count << std::endl;
        return 1;
    }
    std::cerr << "done!\n" << std::endl;
    return 0;
}
