// bin/tags_in_regions -- drop-in for src/tags_in_regions.cpp (SURVEY.md
// 3.4, 8(f)3): counts extra samples' tags inside an existing region table.
//
// The reference walks one cursor per sample through that sample's stream,
// region by region (src/tags_in_regions.cpp:181-195; quirk Q12: the count
// loop has no strand check).  Here every stream is decoded once (the
// parallel wiggle lexer), its prefix sums and skip tables are built on the
// GPU, and the device answers every (region, sample) pair as if the cursor
// started at the stream's first record (up_tir_query).  The host then walks
// the cursors: a region whose device answer starts at or after the cursor is
// exactly the reference's (nothing between the cursor and that start
// qualifies), and only the others -- regions out of order, a forward region
// after the cursor passed into the reverse track, unsorted streams -- are
// walked record by record from the cursor.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <iostream>
#include <memory>
#include <thread>

#include "cli.hpp"
#include "unipeak_hip.h"
#include "wigio.hpp"
#include "gzio.hpp"

using namespace unipeak;

namespace {

struct RegionRow {
    std::string text;
    uint32_t contig, left, right;
    bool fwd;
};

// one sample's records as readAlign() returns them, from the cursor's first
// record on; `complete` false: reading record n raised an input error (the
// reference reports it only if a cursor ever needs that record)
struct Records {
    std::vector<uint64_t> key;
    std::vector<uint32_t> cnt;
    std::vector<uint8_t> fwd;
    bool complete = true;
    void push(const Tag &t) {
        key.push_back((uint64_t)t.contig << 32 | t.first);
        cnt.push_back(t.count);
        fwd.push_back(t.forward ? 1 : 0);
    }
};

void serial_rest(SampleStream &s, Records &out) {
    for (const Align *a = &s.read_align(); a->count != 0; a = &s.read_align())
        out.push(Tag{a->contig, a->first, a->count, a->forward});
}

void decode(SampleStream &s, unsigned threads, Records &out) {
    t_defer_errors = true;
    const Align a0 = s.last();
    if (a0.count != 0) {
        out.push(Tag{a0.contig, a0.first, a0.count, a0.forward});
        bool parallel = false;
        std::vector<Tag> rest;
        try {
            parallel = s.decode_rest(rest, threads);
        } catch (const DeferredError &) {
            // the parallel decode keeps nothing on an error: find the
            // records before it with a serial pass over a fresh stream
            std::unique_ptr<SampleStream> again = s.reopen();
            out = Records();
            try {
                again->read_align();
                out.push(Tag{a0.contig, a0.first, a0.count, a0.forward});
                serial_rest(*again, out);
            } catch (const DeferredError &) {
                out.complete = false;
            }
            t_defer_errors = false;
            return;
        }
        if (parallel) {
            out.key.reserve(rest.size() + 1);
            out.cnt.reserve(rest.size() + 1);
            out.fwd.reserve(rest.size() + 1);
            for (const Tag &t : rest) out.push(t);
        } else {
            try {
                serial_rest(s, out);
            } catch (const DeferredError &) {
                out.complete = false;
            }
        }
    }
    t_defer_errors = false;
}

}  // namespace

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
    // the HIP runtime starts while the streams are decoded
    int ndev = 0;
    std::vector<up_tir *> dev;
    std::thread warm([&] {
        ndev = std::min<int>(cli_device_count(), (int)files.size());
        dev.assign(std::max(ndev, 0), nullptr);
        for (int d = 0; d < ndev; ++d)
            if (up_tir_open(cli_physical_device(d), &dev[d]) != UP_OK) dev[d] = nullptr;
    });
    const size_t S = files.size();
    std::vector<Records> rec(S);
    {
        const unsigned T = ingest_threads();
        const unsigned per = std::max(1u, T / (unsigned)S);
        std::atomic<size_t> next{0};
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < std::min<size_t>(S, T); ++t)
            pool.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < S;) decode(*st[i], per, rec[i]);
            });
        for (auto &th : pool) th.join();
    }
    LineReader rin(in_name);
    std::string o;
    std::string line = rin.read();
    while (line.empty() || line[0] == '#') {  // copy the previous header
        o += line + "\n";
        line = rin.read();
    }
    if (line[0] != '\t') {
        warm.join();
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
    // the region rows up to the first malformed one; the reference reports
    // that line only after walking the cursors through the rows before it
    std::vector<RegionRow> regs;
    std::string row_error;
    while (rin.good()) {
        const std::string l = rin.read();
        if (l.empty()) continue;
        const std::string bad_format = "error: bad format in " + in_name + " line " + std::to_string(rin.line_no()) + "\n\n";
        const size_t colon = l.find_first_of(':'), dash = l.find_first_of('-'), tab = l.find_first_of('\t');
        if (tab == std::string::npos || colon == std::string::npos || dash == std::string::npos ||
            dash > tab || colon > dash) {
            row_error = bad_format;
            break;
        }
        const uint32_t contig = ct.index(l.substr(0, colon));
        if (contig == ct.size()) {
            row_error = "error: contig not in table in " + in_name + " line " + std::to_string(rin.line_no()) + "\n\n";
            break;
        }
        uint64_t a, b;
        if (!lex_uint(l.substr(colon + 1, dash - colon - 1), 0xFFFFFFFFull, &a) ||
            !lex_uint(l.substr(dash + 1, tab - dash - 1), 0xFFFFFFFFull, &b)) {
            row_error = bad_format;
            break;
        }
        const bool fwd = b >= a;
        if (!fwd && !directional) {
            row_error = "error: reverse regions in non-directional analysis\n\n";
            break;
        }
        const uint32_t lo = (uint32_t)(fwd ? a : b), hi = (uint32_t)(fwd ? b : a);
        // (the reference's overlap check never fires: lastContig is never updated)
        regs.push_back(RegionRow{l, contig, lo < ext ? 0 : lo - ext, hi + ext, fwd});
    }
    bool all_complete = true;
    for (const Records &x : rec) all_complete = all_complete && x.complete;
    if (!row_error.empty() && all_complete) {  // no stream can fail before that row
        warm.join();
        for (up_tir *h : dev)
            if (h) up_tir_close(h);
        std::cerr << row_error;
        return 1;
    }
    warm.join();
    if (ndev < 1) fatal("no HIP device available (the GPU path has no CPU fallback)");
    for (int d = 0; d < ndev; ++d)
        if (!dev[d]) fatal("could not open HIP device " + std::to_string(d));
    // device answers: samples dealt to the devices round-robin
    const size_t R = regs.size();
    std::vector<uint32_t> qfirst(R * S), qend(R * S), qhits(R * S);
    {
        std::vector<uint32_t> rc(R), rl(R), rr(R);
        std::vector<uint8_t> rf(R);
        for (size_t r = 0; r < R; ++r) {
            rc[r] = regs[r].contig;
            rl[r] = regs[r].left;
            rr[r] = regs[r].right;
            rf[r] = regs[r].fwd;
        }
        std::vector<std::thread> pool;
        std::vector<int> rcode(ndev, UP_OK);
        for (int d = 0; d < ndev; ++d)
            pool.emplace_back([&, d] {
                std::vector<size_t> mine;
                for (size_t i = d; i < S; i += ndev) mine.push_back(i);
                int e = UP_OK;
                for (size_t k = 0; k < mine.size() && e == UP_OK; ++k) {
                    const Records &x = rec[mine[k]];
                    e = up_tir_set_stream(dev[d], (uint32_t)k, x.key.size(), x.key.data(), x.cnt.data(),
                                          x.fwd.data());
                }
                std::vector<uint32_t> f(R * mine.size()), en(R * mine.size()), h(R * mine.size());
                if (e == UP_OK && R)
                    e = up_tir_query(dev[d], (uint32_t)mine.size(), R, rc.data(), rl.data(), rr.data(),
                                     rf.data(), f.data(), en.data(), h.data());
                for (size_t r = 0; r < R && e == UP_OK; ++r)
                    for (size_t k = 0; k < mine.size(); ++k) {
                        qfirst[r * S + mine[k]] = f[r * mine.size() + k];
                        qend[r * S + mine[k]] = en[r * mine.size() + k];
                        qhits[r * S + mine[k]] = h[r * mine.size() + k];
                    }
                rcode[d] = e;
            });
        for (auto &th : pool) th.join();
        for (int d = 0; d < ndev; ++d) {
            if (rcode[d] != UP_OK) fatal(std::string("tags_in_regions on the GPU failed: ") + up_strerror(rcode[d]));
            up_tir_close(dev[d]);
        }
    }
    // the cursors (tags_in_regions.cpp:183-195), one per sample
    std::vector<uint32_t> hits(R * S);
    std::vector<uint64_t> tir(S, 0);
    std::vector<size_t> fail_at(S, R);  // first region whose walk needs an unreadable record
    {
        std::atomic<size_t> next{0};
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < std::min<size_t>(S, ingest_threads()); ++t)
            pool.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < S;) {
                    const Records &x = rec[i];
                    const uint32_t n = (uint32_t)x.key.size();
                    uint32_t p = 0;  // the record the cursor holds (n: none)
                    for (size_t r = 0; r < R; ++r) {
                        const RegionRow &g = regs[r];
                        const size_t q = r * S + i;
                        uint32_t s = qfirst[q], e = qend[q], h = qhits[q];
                        if (s == UP_TIR_HOST || p > s) {
                            const uint64_t kl = (uint64_t)g.contig << 32 | g.left;
                            const uint64_t kr = (uint64_t)g.contig << 32 | g.right;
                            for (s = p; s < n && !(x.fwd[s] == (uint8_t)g.fwd && x.key[s] >= kl); ++s) {}
                            h = 0;
                            for (e = s; e < n && (x.key[e] >> 32) == g.contig && x.key[e] <= kr; ++e)
                                h += x.cnt[e];
                        }
                        if (!x.complete && (s == n || e == n)) {  // the reference reads record n here
                            fail_at[i] = r;
                            break;
                        }
                        hits[q] = h;
                        tir[i] += h;
                        p = e;
                    }
                }
            });
        for (auto &th : pool) th.join();
    }
    // an input error the reference meets: replay that stream serially to it
    // (the first failing region, then sample, in the reference's order)
    size_t bad = S, bad_r = R;
    for (size_t i = 0; i < S; ++i)
        if (fail_at[i] < bad_r) bad_r = fail_at[i], bad = i;
    if (bad < S) {
        std::unique_ptr<SampleStream> s = st[bad]->reopen();
        while (s->read_align().count != 0) {}  // exits through the reference's error report
        fatal("internal: an input error of " + files[bad] + " did not reproduce");
    }
    if (!row_error.empty()) {
        std::cerr << row_error;
        return 1;
    }
    for (size_t r = 0; r < R; ++r) {
        o += regs[r].text;
        for (size_t i = 0; i < S; ++i) o += "\t" + fmt_lexical(hits[r * S + i]);
        o += "\n";
    }
    FILE *out = out_name == "stdout" ? stdout : open_output(out_name);
    if (!out) { std::cerr << "error: could not write " << out_name << std::endl << std::endl; return 1; }
    std::fwrite(o.data(), 1, o.size(), out);
    if (out != stdout) std::fclose(out); else std::fflush(stdout);
    std::cerr << R << " in " << in_name << std::endl << "tags in regions:" << std::endl;
    for (size_t i = 0; i < st.size(); ++i) {
        char pct[64];
        std::snprintf(pct, sizeof pct, "%.1f", 100 * (double)tir[i] / (double)st[i]->expected_tags());
        std::cerr << "  " << st[i]->expt_name() << ": " << tir[i] << " (" << pct << "%)" << std::endl;
    }
    std::cerr << "\nDone!\n" << std::endl;
    return 0;
}
