// bin/regions -- drop-in for the reference's src/regions.cpp (call stack
// SURVEY.md 3.1/3.2): same flags, headers, row format, emission order and
// stderr summary.  Parsing and the stream merge run on the host; the KDE,
// threshold scan, segmentation and region statistics run on MI355X through
// include/unipeak_hip.h.
#include <cmath>
#include <cstdio>
#include <iostream>
#include <memory>
#include <sstream>

#include "cli.hpp"
#include "engine.hpp"
#include "wigio.hpp"
#include "gzio.hpp"

using namespace unipeak;

int main(int argc, char **argv) {
    ArgParser ap({{"q", "quiet", true, false},          {"D", "non-directional", true, false},
                  {"a", "assembly", false, false},      {"n", "name", false, false},
                  {"w", "wig", false, false},           {"m", "mappable", false, false},
                  {"t", "hitThreshold", false, false},  {"y", "corr", true, false},
                  {"u", "corrThreshold", false, false}, {"k", "kurtosisThreshold", false, false},
                  {"r", "regionThreshold", false, false}, {"z", "coeff", false, false},
                  {"b", "bandwidth", false, false},     {"i", "mismatches", false, false},
                  {"l", "length", false, false},        {"s", "shift", false, false},
                  {"p", "prob", false, false},          {"e", "exclude", false, false},
                  {"f", "peaks", true, false},          {"o", "out", false, true},
                  {"c", "contig", false, true}});
    ap.parse(argc, argv);
    PhaseTimer timer;
    const std::vector<std::string> files = ap.files();
    if (files.empty()) {
        std::cerr << "error: Required argument missing for arg alignment filenames" << std::endl << std::endl;
        return 1;
    }
    const bool quiet = ap.on("q");
    const bool directional = !ap.on("D");
    const std::string profile = ap.str("w");
    uint32_t mappable = (uint32_t)ap.uint("m", 0, 0xFFFFFFFFull);
    double hit_thr = ap.dbl("t", 10);
    bool out_corrs = ap.on("y");
    double corr_thr = ap.dbl("u", 0.3);
    const double kurt_thr = ap.dbl("k", 50);
    const double region_thr = ap.dbl("r", 25);
    const std::string coeff_str = ap.str("z");
    const uint16_t bw = (uint16_t)ap.uint("b", 50, 0xFFFF);
    const uint16_t use_len = (uint16_t)ap.uint("l", 0, 0xFFFF);
    const std::string offset_str = ap.str("s");
    const std::string control_str = ap.str("e");
    const bool out_peaks = ap.on("f");
    const std::string out_name = ap.str("o"), ct_name = ap.str("c");
    const std::string assembly = ap.str("a");
    std::string track_name = ap.str("n");
    if (!profile.empty() && track_name.empty()) track_name = fname_prefix(profile);  // regions.cpp:103

    if (directional) {  // regions.cpp:104-109
        if (corr_thr != 0.3) std::cerr << "warning: correlation threshold is not used on strand-specific analysis" << std::endl;
        corr_thr = -1;
        if (out_corrs) std::cerr << "warning: strand correlations are not calculated for strand-specific analysis" << std::endl;
        out_corrs = false;
    }
    // offsets, regions.cpp:111-127
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
    // controls, regions.cpp:129-150
    std::vector<uint8_t> control(files.size(), 0);
    if (!control_str.empty()) {
        for (const std::string &t : split_csv(control_str)) {
            int16_t v;
            if (!lex_short(t, &v)) { std::cerr << "error: bad control index\n" << std::endl; return 1; }
            const uint16_t idx = (uint16_t)v;
            if (idx == 0) { std::cerr << "error: bad control index (first sample is 1)\n" << std::endl; return 1; }
            if (idx > files.size()) { std::cerr << "error: bad control index (greater than number of samples)\n" << std::endl; return 1; }
            control[idx - 1] = 1;
        }
    }
    uint16_t n_control = 0;
    for (uint8_t c : control) n_control += c;
    hit_thr *= (double)(files.size() - n_control);  // regions.cpp:155
    // coefficients, regions.cpp:157-180
    std::vector<double> coeffs;
    bool prop = false;
    if (!coeff_str.empty()) {
        if (coeff_str == "p") prop = true;
        else {
            for (const std::string &t : split_csv(coeff_str)) {
                double v;
                if (!lex_double(t, &v)) { std::cerr << "error: bad coeff argument\n" << std::endl; return 1; }
                coeffs.push_back(v);
            }
            if (coeffs.size() != files.size() - n_control) {
                std::cerr << "error: wrong number of coeff arguments\nmust have same number as non-control alignment files\n" << std::endl;
                return 1;
            }
        }
    }
    const ContigTable ct = ContigTable::parse(ct_name);
    prewarm_devices(env_gpus());

    // input streams, regions.cpp:184-202
    std::vector<std::unique_ptr<SampleStream>> st;
    std::vector<SampleStream *> sp;
    uint64_t nc_tags = 0, tot_tags = 0;
    std::cerr << "reading alignment files..." << std::endl;
    for (size_t i = 0, oi = 0; i < files.size(); ++i) {
        const int16_t off = offsets.empty() ? 0 : offsets[oi];
        st.emplace_back(new SampleStream(files[i], &ct, off, use_len, !directional));
        sp.push_back(st.back().get());
        const uint64_t tags = st.back()->expected_tags();
        if (!control[i]) nc_tags += tags;
        tot_tags += tags;
        st.back()->read_align();
        std::cerr << "  " << st.back()->expt_name() << ": " << tags << " tags" << std::endl;
        if (offsets.size() > 1) ++oi;
    }
    // background, regions.cpp:204-213
    if (mappable == 0) mappable = ct.genome_size();
    std::cerr << tot_tags << " usable tags";
    if (nc_tags != tot_tags) std::cerr << ", " << nc_tags << " not from negative controls,";
    std::cerr << " at " << mappable << " mappable positions" << std::endl;
    double background = (double)nc_tags / (double)mappable;
    if (directional) background /= 2;
    std::cerr << "using background = " << background << " tags/position";
    if (directional) std::cerr << " on each strand";
    std::cerr << std::endl;
    // coefficients, regions.cpp:215-229 (quirk Q6 in the explicit branch)
    if (prop) {
        for (size_t i = 0; i < files.size(); ++i)
            if (!control[i])
                coeffs.push_back((double)nc_tags / ((double)sp[i]->expected_tags() * (double)(files.size() - n_control)));
    } else if (!coeffs.empty()) {
        double scaled = 0;
        for (size_t i = 0; i < coeffs.size() && i < files.size(); ++i)
            if (!control[i]) scaled += coeffs[i] * (double)sp[i]->expected_tags();
        for (double &c : coeffs) c *= (double)nc_tags / scaled;
    }

    // header, regions.cpp:234-302
    std::ostringstream h;
    for (const std::string &f : files) h << "# align_file=" << f << "\n";
    if (!offsets.empty()) {
        if (offsets.size() == 1) h << "# shift=" << offsets[0] << "\n";
        else {
            h << "# shifts=";
            for (size_t i = 0; i + 1 < offsets.size(); ++i) h << offsets[i] << ",";
            h << offsets.back() << "\n";
        }
    }
    h << "# contig_table=" << ct_name << "\n";
    h << "# bandwidth=" << bw << "\n";
    if (files.size() > 1) {
        h << "# tags=" << sp[0]->expected_tags();
        for (size_t i = 1; i < files.size(); ++i) h << "," << sp[i]->expected_tags();
        h << "\n";
    }
    if (n_control > 0) {
        h << "# control=";
        bool first = true;
        for (size_t i = 0; i < control.size(); ++i)
            if (control[i]) { if (!first) h << ","; first = false; h << i + 1; }
        h << "\n";
    }
    if (!coeffs.empty()) {
        h << "# coeffs=" << coeffs[0];
        for (size_t i = 1; i < coeffs.size(); ++i) h << "," << coeffs[i];
        h << "\n";
    }
    h << "# total_tags=" << nc_tags << "\n";
    h << "# background=" << background << "\n";
    ProfileSink prof;
    if (!profile.empty()) {  // regions.cpp:276-284: header first, profile as positions retire
        prof.fp = profile == "stdout" ? stdout : open_output(profile);
        if (!prof.fp) { std::cerr << "error: could not write " << profile << std::endl << std::endl; exit_now(1); }
        std::setvbuf(prof.fp, nullptr, _IOFBF, 1 << 22);
        prof.ct = &ct;
        prof.directional = directional;
        prof.name = track_name;
        prof.assembly = assembly;
        const std::string hs = h.str();
        std::fwrite(hs.data(), 1, hs.size(), prof.fp);
    }
    std::string table = h.str();
    table += "# region_threshold=" + fmt_lexical(region_thr) + "\n";
    table += "# kurtosis_threshold=" + fmt_lexical(kurt_thr) + "\n";
    table += "# corr_threshold=" + fmt_lexical(corr_thr) + "\n";
    table += "# hit_threshold=" + fmt_lexical(hit_thr) + "\n";
    if (out_peaks) table += "\tpeak";
    if (out_corrs) table += "\tcorrelation";
    table += "\tkurtosis";
    for (SampleStream *s : sp) table += "\t" + s->expt_name();
    table += "\n";

    std::cerr << "calling enriched regions..." << std::endl;
    PassResult pr;
    timer.mark("open");
    build_units(sp, ct, directional, bw, control, coeffs, quiet, pr);
    maybe_dump_units(pr, sp);
    timer.mark("ingest");
    EngineParams ep;
    ep.p.bw = bw;
    ep.p.n_samples = (uint16_t)files.size();
    ep.p.nondir = directional ? 0 : 1;
    ep.p.background = background;
    ep.p.region_thr = region_thr;
    ep.p.kurt_thr = kurt_thr;
    ep.p.corr_thr = corr_thr;
    ep.p.hit_thr = hit_thr;
    ep.p.want_corr = (!directional && (corr_thr > -1 || out_corrs)) ? 1 : 0;
    ep.control = control;
    ep.coeffs = coeffs;
    ep.ngpus = env_gpus();
    ep.profile = prof.fp != nullptr;
    run_units(ep, pr);
    timer.mark("gpu");
    if (prof.fp) {
        write_profile(pr, bw, prof);
        if (prof.fp != stdout) std::fclose(prof.fp); else std::fflush(stdout);
        timer.mark("profile");
    }

    // emission in the reference's order (Q2-Q4); Q3 drops final-flush regions
    const std::vector<Emitted> em = order_candidates(pr, bw, false);
    const size_t S = files.size();
    uint64_t n_pass = 0, n_rej = 0;
    std::vector<uint64_t> tir(S, 0);
    for (const Emitted &e : em) {
        const up_region &r = e.c->r;
        if (!r.accepted) { ++n_rej; continue; }
        ++n_pass;
        for (size_t s = 0; s < S; ++s) tir[s] += e.c->counts[s];
        if (!e.written) continue;
        const UnitBuild &u = pr.units[e.c->unit_index];
        std::string row = ct.name(u.contig) + ":";
        const uint64_t left = r.left, right = r.right;
        row += e.forward_label ? std::to_string(left) + "-" + std::to_string(right)
                               : std::to_string(right) + "-" + std::to_string(left);
        if (out_peaks) row += "\t" + std::to_string(r.peak);
        if (out_corrs) {
            const uint32_t n = r.right - r.left + 1;
            // Region::strandCorr returns quiet_NaN ("nan") for short regions;
            // a computed 0/0 is x86's default NaN ("-nan")
            row += "\t" + (std::isnan(r.corr) ? std::string(n > 3 ? "-nan" : "nan") : fmt_ostream(r.corr));
        }
        row += "\t" + (std::isnan(r.kurtosis) ? std::string("-nan") : fmt_fixed2(r.kurtosis));
        for (size_t s = 0; s < S; ++s) row += "\t" + std::to_string(e.c->counts[s]);
        row += "\n";
        table += row;
    }
    FILE *out = out_name == "stdout" ? stdout : open_output(out_name);
    if (!out) { std::cerr << "error: could not write " << out_name << std::endl << std::endl; exit_now(1); }
    std::fwrite(table.data(), 1, table.size(), out);
    if (out != stdout) std::fclose(out); else std::fflush(stdout);
    timer.mark("table");

    if (!quiet) {  // per-pass progress lines, regions.cpp:312-384, printed after the run
        std::vector<uint64_t> per(pr.units.size(), 0);
        for (const Emitted &e : em)
            if (e.c->r.accepted) per[e.c->unit_index]++;
        uint32_t it = 0;
        bool fwd = true;
        for (uint32_t c = 0; c < ct.size();) {
            uint64_t fr = 0, rr = 0;
            for (size_t k = 0; k < pr.units.size(); ++k)
                if (pr.units[k].iteration == it) (pr.units[k].buffer == 0 ? fr : rr) += per[k];
            std::cerr << "  " << ct.name(c) << (directional ? (fwd ? "+" : "-") : "") << "... ";
            if (fwd) {
                std::cerr << fr << std::endl;
                if (directional && rr > 0) std::cerr << "  " << ct.name(c) << "-... " << rr << std::endl;
            } else {
                std::cerr << rr << std::endl;
            }
            ++c;
            ++it;
            if (directional && c == ct.size() && fwd) { c = 0; fwd = false; }
        }
    }
    std::cerr << n_pass << " regions passed filters, " << n_rej << " rejected" << std::endl;
    std::cerr << "tags in regions:" << std::endl;
    for (size_t i = 0; i < S; ++i) {
        SampleStream &s = *sp[i];
        if (s.confident() + s.out_of_bounds() != s.expected_tags())
            std::cerr << "  warning: expected " << s.expected_tags() << " tags in " << s.expt_name()
                      << " but found " << s.confident() << "; results inaccurate" << std::endl;
        char pct[64];
        std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)tir[i] / (double)s.confident());
        std::cerr << "  " << s.expt_name() << ": " << tir[i] << " (" << pct << "%)" << std::endl;
    }
    std::cerr << "\nAll done!\n" << std::endl;
    release_devices();
    return 0;
}
