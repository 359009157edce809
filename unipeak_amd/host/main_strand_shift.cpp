// bin/strand_shift -- drop-in for src/strand_shift.cpp.
// The region call (one nondirectional buffer) and the strandCorr(shift)
// table run on MI355X; the reference's std::sort by Region::sum() is
// applied on the host to the regions in the reference's push order, so tie
// order (quirk Q15) follows the same libstdc++ algorithm.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <memory>

#include "cli.hpp"
#include "engine.hpp"
#include "wigio.hpp"
#include "gzio.hpp"

using namespace unipeak;

int main(int argc, char **argv) {
    ArgParser ap({{"m", "mappable", false, false},       {"t", "hitThreshold", false, false},
                  {"u", "corrThreshold", false, false},  {"k", "kurtosisThreshold", false, false},
                  {"r", "regionThreshold", false, false}, {"b", "bandwidth", false, false},
                  {"g", "testRegions", false, false},    {"x", "maxShift", false, false},
                  {"n", "minShift", false, false},       {"i", "mismatches", false, false},
                  {"l", "length", false, false},         {"s", "shift", false, false},
                  {"p", "prob", false, false},           {"o", "out", false, false},
                  {"c", "contigs", false, true}});
    ap.parse(argc, argv);
    const std::vector<std::string> files = ap.files();
    if (files.empty()) {
        std::cerr << "error: Required argument missing for arg alignment filenames" << std::endl << std::endl;
        return 1;
    }
    uint32_t mappable = (uint32_t)ap.uint("m", 0, 0xFFFFFFFFull);
    const uint32_t hit_thr = (uint32_t)ap.uint("t", 10, 0xFFFFFFFFull);
    const double corr_thr = ap.dbl("u", 0.3);
    const double kurt_thr = ap.dbl("k", 50);
    const double region_thr = ap.dbl("r", 25);
    const uint16_t bw = (uint16_t)ap.uint("b", 50, 0xFFFF);
    const uint16_t n_test = (uint16_t)ap.uint("g", 1000, 0xFFFF);
    const uint16_t max_shift = (uint16_t)ap.uint("x", 150, 0xFFFF);
    const uint16_t min_shift = (uint16_t)ap.uint("n", 25, 0xFFFF);
    const uint16_t use_len = (uint16_t)ap.uint("l", 0, 0xFFFF);
    const std::string offset_str = ap.str("s"), out_name = ap.str("o"), ct_name = ap.str("c");

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
    prewarm_devices(env_gpus());
    std::vector<std::unique_ptr<SampleStream>> st;
    std::vector<SampleStream *> sp;
    uint64_t total = 0;
    std::cerr << "reading alignment files..." << std::endl;
    for (size_t i = 0, oi = 0; i < files.size(); ++i) {
        const int16_t off = offsets.empty() ? 0 : offsets[oi];
        st.emplace_back(new SampleStream(files[i], &ct, off, use_len, true));
        sp.push_back(st.back().get());
        const uint64_t tags = st.back()->expected_tags();
        total += tags;
        st.back()->read_align();
        std::cerr << "  " << st.back()->expt_name() << ": " << tags << " tags" << std::endl;
        if (offsets.size() > 1) ++oi;
    }
    if (mappable == 0) mappable = ct.genome_size();
    std::cerr << total << " usable tags at " << mappable << " mappable positions" << std::endl;
    const double background = (double)total / (double)mappable;
    std::cerr << "using background = " << background << " tags/position" << std::endl;
    std::cerr << "calling enriched regions for shift calibration... " << std::flush;

    const size_t S = files.size();
    std::vector<uint8_t> control(S, 0);
    PassResult pr;
    build_units(sp, ct, false, bw, control, {}, true, pr);
    maybe_dump_units(pr, sp);
    EngineParams ep;
    ep.p.bw = bw;
    ep.p.n_samples = (uint16_t)S;
    ep.p.nondir = 1;
    ep.p.background = background;
    ep.p.region_thr = region_thr;
    ep.p.kurt_thr = kurt_thr;
    ep.p.corr_thr = -1;  // strand_shift.cpp:142
    ep.p.hit_thr = (double)hit_thr;  // not scaled by S (quirk Q13)
    ep.p.want_corr = 0;
    ep.control = control;
    ep.ngpus = env_gpus();
    run_units(ep, pr);
    const std::vector<Emitted> em = order_candidates(pr, bw, true);
    std::cerr << em.size() << " found\n";

    // std::sort of the push-ordered regions by sum(), descending (:198)
    std::vector<const Candidate *> regs;
    for (const Emitted &e : em) regs.push_back(e.c);
    std::sort(regs.begin(), regs.end(),
              [](const Candidate *a, const Candidate *b) { return a->r.sum > b->r.sum; });
    // strandCorr(0..maxShift) of every region long enough to be tested
    std::vector<const Candidate *> elig;
    for (const Candidate *c : regs)
        if ((uint64_t)(c->r.right - c->r.left + 1) > (unsigned)(2 * max_shift + 3)) elig.push_back(c);
    // per region the first shift with the largest correlation (:209-217),
    // reduced on the GPU -- for the regions the reference's loop reaches:
    // it stops at the n_test-th qualifying one, so the sorted regions go to
    // the device in chunks (the first n_test + n_test/4, then twice what is
    // still missing) until enough qualify or none are left
    uint16_t tested = 0;
    uint64_t tags_in = 0;
    std::vector<uint64_t> freq((size_t)max_shift + 1, 0);
    const size_t W = (size_t)max_shift + 1;
    size_t done = 0;
    while (tested < n_test && done < elig.size()) {
        const size_t want = done == 0 ? (size_t)n_test + n_test / 4 + 16 : 2 * (size_t)(n_test - tested) + 16;
        const size_t m = std::min(want, elig.size() - done);
        std::vector<const Candidate *> chunk(elig.begin() + done, elig.begin() + done + m);
        std::vector<uint16_t> bshift;
        std::vector<double> bcorr;
        shift_best(ep, pr, chunk, max_shift, bshift, bcorr);
        for (size_t k = 0; tested < n_test && k < m; ++k) {
            if (bcorr[k] >= corr_thr) {
                ++freq[bshift[k]];
                tags_in += chunk[k]->r.sum;
                ++tested;
            }
        }
        done += m;
    }
    if (tested == 0) { std::cerr << "error: no regions qualified with given settings" << std::endl << std::endl; exit_now(1); }
    if (tested < n_test) std::cerr << "warning: too few regions qualified with given settings" << std::endl;
    char pct[64];
    std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)tags_in / (double)total);
    std::cerr << "the top " << tested << " qualified regions contained " << tags_in << " tags (" << pct << "%)" << std::endl;

    // smoothed mode, strand_shift.cpp:241-258
    std::vector<double> mk(11);
    up_kernel_weights(5, 1, mk.data());
    std::vector<double> dens(W, 0);
    for (size_t i = 0; i < W; ++i)
        for (int j = 0; j < 11; ++j) {
            const long k = (long)i - 5 + j;
            if (k >= 0 && k < (long)W) dens[k] += (double)freq[i] * mk[j];
        }
    double best_d = 0;
    uint16_t best_shift = 0;
    for (size_t i = min_shift; i < W - 5; ++i)
        if (dens[i] > best_d) { best_shift = (uint16_t)i; best_d = dens[i]; }
    std::cerr << "estimated shift = " << best_shift << std::endl;

    if (!out_name.empty()) {
        std::cerr << "writing output to " << out_name << "... " << std::flush;
        std::string o;
        for (const std::string &f : files) o += "# align_file=" + f + "\n";
        if (!offsets.empty()) {
            if (offsets.size() == 1) o += "# shift=" + fmt_lexical(offsets[0]) + "\n";
            else {
                o += "# shifts=";
                for (size_t i = 0; i + 1 < offsets.size(); ++i) o += fmt_lexical(offsets[i]) + ",";
                o += fmt_lexical(offsets.back()) + "\n";
            }
        }
        o += "# contig_table=" + ct_name + "\n";
        o += "# bandwidth=" + fmt_lexical(bw) + "\n";
        o += "# tags=" + fmt_lexical((double)total) + "\n";
        o += "# background=" + fmt_lexical(background) + "\n";
        o += "# region_threshold=" + fmt_lexical(region_thr) + "\n";
        o += "# kurtosis_threshold=" + fmt_lexical(kurt_thr) + "\n";
        o += "# corr_threshold=" + fmt_lexical(corr_thr) + "\n";
        o += "# hit_threshold=" + fmt_lexical(hit_thr) + "\n";
        o += "# regions_tested=" + fmt_lexical(tested) + "\n";
        o += "# tags_in_regions=" + fmt_lexical((double)tags_in) + "\n";
        o += "# min_shift=" + fmt_lexical(min_shift) + "\n";
        o += "# best_shift=" + fmt_lexical(best_shift) + "\n\n";
        o += "shift\tregions\n";
        for (size_t i = 0; i < W; ++i)
            if (freq[i]) o += fmt_lexical((double)i) + "\t" + fmt_lexical((double)freq[i]) + "\n";
        FILE *out = out_name == "stdout" ? stdout : open_output(out_name);
        if (!out) { std::cerr << "error: could not write " << out_name << std::endl << std::endl; exit_now(1); }
        std::fwrite(o.data(), 1, o.size(), out);
        if (out != stdout) std::fclose(out); else std::fflush(stdout);
    }
    std::cerr << "done!\n" << std::endl;
    release_devices();
    return 0;
}
