// bin/tags_in_regions -- drop-in for src/tags_in_regions.cpp (SURVEY.md
// 3.4): counts extra samples' tags inside an existing region table.  The
// work is a stream merge with the reference's exact skip/count semantics
// (quirk Q12: the count loop has no strand check), so it runs on the host.
#include <cstdio>
#include <iostream>
#include <memory>

#include "cli.hpp"
#include "wigio.hpp"

using namespace unipeak;

int main(int argc, char **argv) {
    ArgParser ap({{"D", "non-directional", true, false}, {"i", "mismatches", false, false},
                  {"l", "length", false, false},         {"s", "shift", false, false},
                  {"p", "prob", false, false},           {"e", "extend", false, false},
                  {"o", "out", false, true},             {"f", "in", false, true},
                  {"c", "contig", false, true}});
    ap.parse(argc, argv);
    const std::vector<std::string> files = ap.files();
    if (files.empty()) {
        std::cerr << "error: Required argument missing for arg alignment filenames" << std::endl << std::endl;
        return 1;
    }
    const bool directional = !ap.on("D");
    const uint16_t use_len = (uint16_t)ap.uint("l", 0, 0xFFFF);
    const std::string offset_str = ap.str("s");
    const uint32_t ext = (uint32_t)ap.uint("e", 0, 0xFFFFFFFFull);
    const std::string out_name = ap.str("o"), in_name = ap.str("f"), ct_name = ap.str("c");
    std::vector<int16_t> offsets;
    if (!offset_str.empty()) {
        for (const std::string &t : split_csv(offset_str)) {
            int16_t v;
            if (!lex_short(t, &v)) { std::cerr << "error: bad offset argument\n" << std::endl; return 1; }
            offsets.push_back(v);
        }
        if (!(offsets.size() == files.size() || offsets.size() == 1)) {
            std::cerr << "error: wrong number of offset arguments\nmust have same number as alignment files or just one\n" << std::endl;
            return 1;
        }
    }
    const ContigTable ct = ContigTable::parse(ct_name);
    std::vector<std::unique_ptr<SampleStream>> st;
    std::cerr << "reading alignment files..." << std::endl;
    for (size_t i = 0, oi = 0; i < files.size(); ++i) {
        const int16_t off = offsets.empty() ? 0 : offsets[oi];
        st.emplace_back(new SampleStream(files[i], &ct, off, use_len, !directional));
        const uint64_t tags = st.back()->expected_tags();
        st.back()->read_align();
        std::cerr << "  " << st.back()->expt_name() << ": " << tags << " tags" << std::endl;
        if (offsets.size() > 1) ++oi;
    }
    LineReader rin(in_name);
    std::string o;
    std::string line = rin.read();
    while (line.empty() || line[0] == '#') {  // copy the previous header
        o += line + "\n";
        line = rin.read();
    }
    if (line[0] != '\t') {
        std::cerr << "error: bad format in " << in_name << " line " << rin.line_no() << "\n\n";
        return 1;
    }
    if (ext != 0) o += "# region_extension=" + fmt_lexical(ext) + "\n";
    for (const std::string &f : files) o += "# extra_align_file=" + f + "\n";
    if (!offsets.empty()) {
        if (offsets.size() == 1) o += "# shift=" + fmt_lexical(offsets[0]) + "\n";
        else {
            o += "# shifts=";
            for (size_t i = 0; i + 1 < offsets.size(); ++i) o += fmt_lexical(offsets[i]) + ",";
            o += fmt_lexical(offsets.back()) + "\n";
        }
    }
    o += line;
    for (auto &s : st) o += "\t" + s->expt_name();
    o += "\n";
    std::cerr << "processing regions... " << std::flush;
    std::vector<uint64_t> tir(files.size(), 0);
    uint64_t nreg = 0;
    while (rin.good()) {
        const std::string l = rin.read();
        if (l.empty()) continue;
        const size_t colon = l.find_first_of(':'), dash = l.find_first_of('-'), tab = l.find_first_of('\t');
        if (tab == std::string::npos || colon == std::string::npos || dash == std::string::npos ||
            dash > tab || colon > dash) {
            std::cerr << "error: bad format in " << in_name << " line " << rin.line_no() << "\n\n";
            return 1;
        }
        const uint32_t contig = ct.index(l.substr(0, colon));
        if (contig == ct.size()) {
            std::cerr << "error: contig not in table in " << in_name << " line " << rin.line_no() << "\n\n";
            return 1;
        }
        uint64_t a, b;
        if (!lex_uint(l.substr(colon + 1, dash - colon - 1), 0xFFFFFFFFull, &a) ||
            !lex_uint(l.substr(dash + 1, tab - dash - 1), 0xFFFFFFFFull, &b)) {
            std::cerr << "error: bad format in " << in_name << " line " << rin.line_no() << "\n\n";
            return 1;
        }
        const bool fwd = b >= a;
        if (!fwd && !directional) {
            std::cerr << "error: reverse regions in non-directional analysis\n\n";
            return 1;
        }
        const uint32_t lo = (uint32_t)(fwd ? a : b), hi = (uint32_t)(fwd ? b : a);
        const uint32_t left = lo < ext ? 0 : lo - ext, right = hi + ext;
        // (the reference's overlap check never fires: lastContig is never updated)
        o += l;
        for (size_t i = 0; i < st.size(); ++i) {
            const Align *al = &st[i]->last();
            while (al->count != 0 && (fwd != al->forward || al->contig < contig ||
                                      (al->contig == contig && al->first < left)))
                al = &st[i]->read_align();
            uint32_t hits = 0;
            while (al->contig == contig && al->first <= right) {  // no strand check (Q12)
                hits += al->count;
                al = &st[i]->read_align();
            }
            o += "\t" + fmt_lexical(hits);
            tir[i] += hits;
        }
        o += "\n";
        ++nreg;
    }
    FILE *out = out_name == "stdout" ? stdout : std::fopen(out_name.c_str(), "wb");
    if (!out) { std::cerr << "error: could not write " << out_name << std::endl << std::endl; return 1; }
    std::fwrite(o.data(), 1, o.size(), out);
    if (out != stdout) std::fclose(out); else std::fflush(stdout);
    std::cerr << nreg << " in " << in_name << std::endl << "tags in regions:" << std::endl;
    for (size_t i = 0; i < st.size(); ++i) {
        char pct[64];
        std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)tir[i] / (double)st[i]->expected_tags());
        std::cerr << "  " << st[i]->expt_name() << ": " << tir[i] << " (" << pct << "%)" << std::endl;
    }
    std::cerr << "\nDone!\n" << std::endl;
    return 0;
}
