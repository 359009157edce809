// bin/wigs2bigwigs -- drop-in for extras/wigs2bigwigs.pl:
// UniPeak wiggle files (tag counts, or the -w density profiles) -> one UCSC
// bigWig file per track, with the track headers to load them printed on
// stdout.  The script pipes each track into UCSC wigToBigWig -clip; this
// writes the bigWig itself (BBI version 4: chromosome B+ tree, zlib-compressed
// varStep sections of up to 1024 items, R-tree index, and zoom levels as
// wigToBigWig builds them), so the pipeline needs no external tool.
//
// Script behaviour kept (extras/wigs2bigwigs.pl:42-75): output root = input
// name minus /.gz$/ or /.bz2$/ then /.wig$/; '#' lines skipped; a track line
// starts "<root><strand>.bw" (strand = the last +/- before a closing quote of
// name="..."), and prints the header with wiggle_0 -> bigWig and
// " bigDataUrl=<prefix><file>"; any other line goes to the current track
// ("error: no track defined at line N" before the first).  wigToBigWig -clip
// behaviour kept: variableStep (span=), fixedStep (start=, step=, span=) and
// bedGraph lines; items past the chromosome end are clipped (dropped when
// they start past it); chromosomes must be in the sizes file.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <string>
#include <vector>

namespace {

[[noreturn]] void die(const std::string &m) {
    std::cerr << m;
    std::exit(1);
}

struct Item {
    uint32_t start, end;
    float value;
};

struct Track {
    std::string out;                              // output file
    std::map<std::string, std::vector<Item>> by;  // chromosome -> items
};

void put32(std::string &b, uint32_t v) { b.append((const char *)&v, 4); }
void put64(std::string &b, uint64_t v) { b.append((const char *)&v, 8); }
void put16(std::string &b, uint16_t v) { b.append((const char *)&v, 2); }
void putf(std::string &b, float v) { b.append((const char *)&v, 4); }
void putd(std::string &b, double v) { b.append((const char *)&v, 8); }
void set64(std::string &b, size_t at, uint64_t v) { std::memcpy(&b[at], &v, 8); }

struct Block {  // one compressed section and its extent
    uint32_t chrom, start, end;
    uint64_t offset, size;
};

// R-tree (cirTree) over the blocks, bottom-up, blockSize children per node
void write_rtree(std::string &f, const std::vector<Block> &blocks, uint32_t block_size, uint32_t items_per_slot) {
    const uint64_t data_end = f.size();
    put32(f, 0x2468ACE0u);
    put32(f, block_size);
    put64(f, blocks.size());
    put32(f, blocks.empty() ? 0 : blocks.front().chrom);
    put32(f, blocks.empty() ? 0 : blocks.front().start);
    put32(f, blocks.empty() ? 0 : blocks.back().chrom);
    uint32_t end_base = 0;
    for (const Block &b : blocks)
        if (b.chrom == blocks.back().chrom) end_base = std::max(end_base, b.end);
    put32(f, end_base);
    put64(f, data_end);
    put32(f, items_per_slot);
    put32(f, 0);
    // levels: level 0 = leaves over the blocks; each parent level groups
    // block_size nodes.  Nodes are written root first.
    struct Node {
        uint32_t c0, s0, c1, s1;
        size_t first, count;  // children in the level below
    };
    std::vector<std::vector<Node>> levels;
    {
        std::vector<Node> leaves;
        for (size_t i = 0; i < blocks.size(); i += block_size) {
            const size_t n = std::min<size_t>(block_size, blocks.size() - i);
            Node nd{blocks[i].chrom, blocks[i].start, blocks[i + n - 1].chrom, 0, i, n};
            for (size_t k = i; k < i + n; ++k)
                if (blocks[k].chrom == nd.c1) nd.s1 = std::max(nd.s1, blocks[k].end);
            leaves.push_back(nd);
        }
        if (leaves.empty()) leaves.push_back(Node{0, 0, 0, 0, 0, 0});
        levels.push_back(leaves);
    }
    while (levels.back().size() > 1) {
        const std::vector<Node> &below = levels.back();
        std::vector<Node> up;
        for (size_t i = 0; i < below.size(); i += block_size) {
            const size_t n = std::min<size_t>(block_size, below.size() - i);
            Node nd{below[i].c0, below[i].s0, below[i + n - 1].c1, 0, i, n};
            for (size_t k = i; k < i + n; ++k)
                if (below[k].c1 == nd.c1) nd.s1 = std::max(nd.s1, below[k].s1);
            up.push_back(nd);
        }
        levels.push_back(up);
    }
    // offsets: root level first, then downwards
    const size_t L = levels.size();
    std::vector<std::vector<uint64_t>> off(L);
    uint64_t at = f.size();
    for (size_t l = L; l-- > 0;) {
        const bool leaf = l == 0;
        for (const Node &nd : levels[l]) {
            off[l].push_back(at);
            at += 4 + nd.count * (leaf ? 32 : 24);
        }
    }
    for (size_t l = L; l-- > 0;) {
        const bool leaf = l == 0;
        for (const Node &nd : levels[l]) {
            f.push_back(leaf ? 1 : 0);
            f.push_back(0);
            put16(f, (uint16_t)nd.count);
            for (size_t k = nd.first; k < nd.first + nd.count; ++k) {
                if (leaf) {
                    const Block &b = blocks[k];
                    put32(f, b.chrom);
                    put32(f, b.start);
                    put32(f, b.chrom);
                    put32(f, b.end);
                    put64(f, b.offset);
                    put64(f, b.size);
                } else {
                    const Node &c = levels[l - 1][k];
                    put32(f, c.c0);
                    put32(f, c.s0);
                    put32(f, c.c1);
                    put32(f, c.s1);
                    put64(f, off[l - 1][k]);
                }
            }
        }
    }
}

// one zoom-level record (bbiSummaryOnDisk): the bases of one bin that hold
// data, and their value statistics
struct Summary {
    uint32_t chrom, start, end, valid;
    float vmin, vmax;
    double sum, sumsq;  // (double in memory, float on disk, as bbiSummary)
};

// the summaries of one zoom level as wigToBigWig builds them
// (bbiAddRangeToSummary): bins of `reduction` bases that start at the first
// item of a run (or continue the previous bin), items split across bin
// edges, clipped at the chromosome's end
std::vector<Summary> summarise(const std::vector<std::vector<Item>> &items, const std::vector<uint32_t> &csize,
                               uint32_t reduction) {
    std::vector<Summary> out;
    for (uint32_t ci = 0; ci < items.size(); ++ci) {
        bool have = false;
        for (const Item &it : items[ci]) {
            uint32_t start = it.start;
            const uint32_t end = std::min(it.end, csize[ci]);
            while (start < end) {
                Summary *sm = have ? &out.back() : nullptr;
                if (!sm || sm->end <= start) {
                    Summary n{};
                    n.chrom = ci;
                    n.start = (!sm || (uint64_t)sm->end + reduction <= start) ? start : sm->end;
                    n.end = (uint32_t)std::min<uint64_t>((uint64_t)n.start + reduction, csize[ci]);
                    n.vmin = n.vmax = it.value;
                    out.push_back(n);
                    have = true;
                    sm = &out.back();
                }
                const uint32_t ov = std::min(end, sm->end) - std::max(start, sm->start);
                sm->valid += ov;
                sm->vmin = std::min(sm->vmin, it.value);
                sm->vmax = std::max(sm->vmax, it.value);
                sm->sum += (double)it.value * ov;
                sm->sumsq += (double)it.value * it.value * ov;
                start += ov;
            }
        }
    }
    return out;
}

void write_bigwig(const Track &t, const std::map<std::string, uint32_t> &sizes) {
    // chromosome ids in name order (the B+ tree's key order)
    std::vector<std::string> names;
    for (const auto &kv : t.by) names.push_back(kv.first);
    std::sort(names.begin(), names.end());
    size_t key_size = 1;
    for (const std::string &n : names) key_size = std::max(key_size, n.size());
    std::vector<std::vector<Item>> sorted(names.size());
    std::vector<uint32_t> csize(names.size());
    uint64_t nitems = 0, bases = 0;
    for (size_t ci = 0; ci < names.size(); ++ci) {
        sorted[ci] = t.by.at(names[ci]);
        std::stable_sort(sorted[ci].begin(), sorted[ci].end(),
                         [](const Item &a, const Item &b) { return a.start < b.start; });
        csize[ci] = sizes.at(names[ci]);
        for (const Item &it : sorted[ci]) bases += it.end - it.start;
        nitems += sorted[ci].size();
    }
    // zoom levels (wigToBigWig: up to 10, each 4x the previous, the first
    // 10x the average item span): a level is kept while it has fewer
    // summaries than the level before it (and than the items themselves)
    std::vector<std::pair<uint32_t, std::vector<Summary>>> zooms;
    if (nitems) {
        uint64_t red = std::max<uint64_t>(1, (bases + nitems / 2) / nitems) * 10;
        size_t prev = nitems;
        for (int z = 0; z < 10 && red < 0xFFFFFFFFull; ++z, red *= 4) {
            std::vector<Summary> sm = summarise(sorted, csize, (uint32_t)red);
            if (sm.empty() || sm.size() >= prev) break;
            prev = sm.size();
            zooms.emplace_back((uint32_t)red, std::move(sm));
        }
    }
    std::string f(64 + 24 * zooms.size(), '\0');  // header and zoom headers, patched at the end
    const uint64_t summary_off = f.size();
    f.append(40, '\0');
    const uint64_t tree_off = f.size();
    const uint32_t nchrom = (uint32_t)names.size();
    if (nchrom > 65535) die("error: too many chromosomes for one B+ tree node\n");
    put32(f, 0x78CA8C91u);
    put32(f, std::max<uint32_t>(nchrom, 1));
    put32(f, (uint32_t)key_size);
    put32(f, 8);
    put64(f, nchrom);
    put64(f, 0);
    f.push_back(1);
    f.push_back(0);
    put16(f, (uint16_t)nchrom);
    for (uint32_t i = 0; i < nchrom; ++i) {
        std::string k = names[i];
        k.resize(key_size, '\0');
        f += k;
        put32(f, i);
        put32(f, sizes.at(names[i]));
    }
    // data: varStep sections of up to 1024 items, span 1 per section run
    const uint64_t data_off = f.size();
    put64(f, 0);  // section count, patched
    std::vector<Block> blocks;
    uint32_t max_raw = 0;
    uint64_t valid = 0;
    double vmin = INFINITY, vmax = -INFINITY, vsum = 0, vsq = 0;
    for (uint32_t ci = 0; ci < nchrom; ++ci) {
        const std::vector<Item> &items = sorted[ci];
        for (size_t i = 0; i < items.size();) {
            // a section: consecutive items with the same span, <= 1024
            const uint32_t span = items[i].end - items[i].start;
            size_t j = i;
            while (j < items.size() && j - i < 1024 && items[j].end - items[j].start == span) ++j;
            std::string raw;
            put32(raw, ci);
            put32(raw, items[i].start);
            put32(raw, items[j - 1].end);
            put32(raw, 0);
            put32(raw, span);
            raw.push_back(2);  // varStep
            raw.push_back(0);
            put16(raw, (uint16_t)(j - i));
            for (size_t k = i; k < j; ++k) {
                put32(raw, items[k].start);
                putf(raw, items[k].value);
                const double v = items[k].value;
                valid += span;
                vmin = std::min(vmin, v);
                vmax = std::max(vmax, v);
                vsum += v * span;
                vsq += v * v * span;
            }
            max_raw = std::max<uint32_t>(max_raw, (uint32_t)raw.size());
            uLongf clen = compressBound(raw.size());
            std::string comp(clen, '\0');
            if (compress2((Bytef *)&comp[0], &clen, (const Bytef *)raw.data(), raw.size(), 6) != Z_OK)
                die("error: compression failed\n");
            comp.resize(clen);
            blocks.push_back(Block{ci, items[i].start, items[j - 1].end, f.size(), clen});
            f += comp;
            i = j;
        }
    }
    set64(f, data_off, blocks.size());
    const uint64_t index_off = f.size();
    write_rtree(f, blocks, 256, 1024);
    // zoom levels: per level a uint32 record count, zlib blocks of up to 1024
    // summaries (one chromosome each), their R-tree
    std::vector<std::pair<uint64_t, uint64_t>> zoff;  // data, index
    for (const auto &zl : zooms) {
        const std::vector<Summary> &sm = zl.second;
        const uint64_t zdata = f.size();
        put32(f, (uint32_t)sm.size());
        std::vector<Block> zb;
        for (size_t i = 0; i < sm.size();) {
            size_t j = i;
            while (j < sm.size() && j - i < 1024 && sm[j].chrom == sm[i].chrom) ++j;
            std::string raw;
            for (size_t k = i; k < j; ++k) {
                put32(raw, sm[k].chrom);
                put32(raw, sm[k].start);
                put32(raw, sm[k].end);
                put32(raw, sm[k].valid);
                putf(raw, sm[k].vmin);
                putf(raw, sm[k].vmax);
                putf(raw, (float)sm[k].sum);
                putf(raw, (float)sm[k].sumsq);
            }
            max_raw = std::max<uint32_t>(max_raw, (uint32_t)raw.size());
            uLongf clen = compressBound(raw.size());
            std::string comp(clen, '\0');
            if (compress2((Bytef *)&comp[0], &clen, (const Bytef *)raw.data(), raw.size(), 6) != Z_OK)
                die("error: compression failed\n");
            comp.resize(clen);
            zb.push_back(Block{sm[i].chrom, sm[i].start, sm[j - 1].end, f.size(), clen});
            f += comp;
            i = j;
        }
        const uint64_t zindex = f.size();
        write_rtree(f, zb, 256, 1024);
        zoff.emplace_back(zdata, zindex);
    }
    put32(f, 0x888FFC26u);  // trailing magic
    // header, zoom headers and total summary
    std::string h;
    put32(h, 0x888FFC26u);
    put16(h, 4);
    put16(h, (uint16_t)zooms.size());
    put64(h, tree_off);
    put64(h, data_off);
    put64(h, index_off);
    put16(h, 0);
    put16(h, 0);
    put64(h, 0);
    put64(h, summary_off);
    put32(h, max_raw);
    put64(h, 0);
    for (size_t z = 0; z < zooms.size(); ++z) {
        put32(h, zooms[z].first);
        put32(h, 0);
        put64(h, zoff[z].first);
        put64(h, zoff[z].second);
    }
    std::memcpy(&f[0], h.data(), h.size());
    std::string s;
    put64(s, valid);
    putd(s, valid ? vmin : 0);
    putd(s, valid ? vmax : 0);
    putd(s, vsum);
    putd(s, vsq);
    std::memcpy(&f[summary_off], s.data(), 40);
    FILE *fp = std::fopen(t.out.c_str(), "wb");
    if (!fp) die("error: " + t.out + ": could not write\n");
    std::fwrite(f.data(), 1, f.size(), fp);
    std::fclose(fp);
}

// Perl's s/<any char><suffix>$// as the script writes its regexes
std::string strip_re(const std::string &s, const std::string &suffix) {
    if (s.size() >= suffix.size() + 1 && s.compare(s.size() - suffix.size(), suffix.size(), suffix) == 0)
        return s.substr(0, s.size() - suffix.size() - 1);
    return s;
}

bool read_lines(const std::string &path, std::vector<std::string> &out) {
    // the Perl script pipes *.bz2 through bunzip2; libbz2 is not in this image
    if (path.size() > 4 && path.compare(path.size() - 4, 4, ".bz2") == 0)
        die("error: " + path + ": bzip2 (.bz2) input is not supported by this build; "
            "decompress it first (bunzip2)\n");
    if (path.size() > 3 && path.compare(path.size() - 3, 3, ".gz") == 0) {
        gzFile g = gzopen(path.c_str(), "rb");
        if (!g) return false;
        std::string cur;
        char buf[1 << 16];
        int k;
        while ((k = gzread(g, buf, sizeof buf)) > 0) cur.append(buf, k);
        gzclose(g);
        size_t b = 0;
        for (size_t i = 0; i < cur.size(); ++i)
            if (cur[i] == '\n') { out.push_back(cur.substr(b, i - b + 1)); b = i + 1; }
        if (b < cur.size()) out.push_back(cur.substr(b));
        return true;
    }
    FILE *fp = std::fopen(path.c_str(), "rb");
    if (!fp) return false;
    std::string cur;
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, fp)) > 0) cur.append(buf, k);
    std::fclose(fp);
    size_t b = 0;
    for (size_t i = 0; i < cur.size(); ++i)
        if (cur[i] == '\n') { out.push_back(cur.substr(b, i - b + 1)); b = i + 1; }
    if (b < cur.size()) out.push_back(cur.substr(b));
    return true;
}

}  // namespace

int main(int argc, char **argv) {
    std::string prefix = "http://www.stanford.edu/~yourusername/", sizes_path = "somepath/somefile.chrom.sizes";
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&](const std::string &name) -> bool {
            if (a == "--" + name || a == "-" + name) {
                if (i + 1 >= argc) die("error: bad arguments\n");
                const std::string v = argv[++i];
                if (name == "prefix") prefix = v;
                else if (name == "sizes") sizes_path = v;
                return true;
            }
            if (a.rfind("--" + name + "=", 0) == 0) {
                const std::string v = a.substr(name.size() + 3);
                if (name == "prefix") prefix = v;
                else if (name == "sizes") sizes_path = v;
                return true;
            }
            return false;
        };
        if (val("prefix") || val("sizes") || val("executable")) continue;  // --executable: not needed
        if (a.size() > 1 && a[0] == '-') die("error: bad arguments\n");
        files.push_back(a);
    }
    if (argc == 1)
        die(std::string("\nUsage: ") + argv[0] + " [arguments] file1.wig file2.wig file3.wig.gz ...\n\n"
            "Optional arguments:\n  --prefix <filename prefix>  prefix for URLs\n"
            "  --sizes <filename>          path to chrom.sizes file\n"
            "  --executable <filename>     path to executable\n");
    if (files.empty()) die("error: no input files\n");
    std::map<std::string, uint32_t> sizes;
    {
        std::vector<std::string> lines;
        if (!read_lines(sizes_path, lines)) die("error: could not read " + sizes_path + "\n");
        for (const std::string &l : lines) {
            char name[4096];
            unsigned long long sz;
            if (std::sscanf(l.c_str(), "%4095s %llu", name, &sz) == 2) sizes[name] = (uint32_t)sz;
        }
    }
    for (const std::string &in : files) {
        std::string root = strip_re(strip_re(strip_re(in, "gz"), "bz2"), "wig");
        std::vector<std::string> lines;
        if (!read_lines(in, lines)) die("error reading " + in + ": No such file or directory\n");
        std::vector<Track> tracks;
        // wig parser state of the current track
        std::string chrom;
        int mode = 0;  // 0 bedGraph, 1 variableStep, 2 fixedStep
        uint32_t span = 1, fstart = 0, fstep = 1;
        for (size_t ln = 0; ln < lines.size(); ++ln) {
            const std::string &raw = lines[ln];
            if (!raw.empty() && raw[0] == '#') continue;
            if (raw.compare(0, 5, "track") == 0) {
                std::string header = raw;
                if (!header.empty() && header.back() == '\n') header.pop_back();
                std::string strand;
                const size_t nq = header.find("name=\"");
                if (nq != std::string::npos) {  // name=".+([+-])" : the last [+-]" after one character
                    for (size_t k = header.size(); k-- > nq + 7;)
                        if ((header[k] == '+' || header[k] == '-') && k + 1 < header.size() && header[k + 1] == '"') {
                            strand = header.substr(k, 1);
                            break;
                        }
                }
                tracks.push_back(Track{root + strand + ".bw", {}});
                chrom.clear();
                mode = 0;
                const size_t w = header.find("wiggle_0");
                if (w != std::string::npos) header.replace(w, 8, "bigWig");
                std::cout << header << " bigDataUrl=" << prefix << tracks.back().out << "\n";
                continue;
            }
            if (raw.empty()) continue;
            if (tracks.empty()) die("error: no track defined at line " + std::to_string(ln + 1) + "\n");
            std::string l = raw;
            while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
            if (l.empty()) continue;
            Track &t = tracks.back();
            auto field = [&](const char *key) -> std::string {
                const size_t k = l.find(key);
                if (k == std::string::npos) return "";
                const size_t b = k + std::strlen(key);
                const size_t e = l.find_first_of(" \t", b);
                return l.substr(b, e == std::string::npos ? std::string::npos : e - b);
            };
            auto add = [&](const std::string &c, uint64_t s, uint64_t e, double v) {
                const auto sz = sizes.find(c);
                if (sz == sizes.end())
                    die("error: " + c + " is not found in chromosome sizes file " + sizes_path + "\n");
                if (s >= sz->second) return;  // -clip
                if (e > sz->second) e = sz->second;
                t.by[c].push_back(Item{(uint32_t)s, (uint32_t)e, (float)v});
            };
            if (l.compare(0, 12, "variableStep") == 0) {
                mode = 1;
                chrom = field("chrom=");
                const std::string sp = field("span=");
                span = sp.empty() ? 1 : (uint32_t)std::strtoul(sp.c_str(), nullptr, 10);
            } else if (l.compare(0, 9, "fixedStep") == 0) {
                mode = 2;
                chrom = field("chrom=");
                const std::string sp = field("span="), st = field("step="), s0 = field("start=");
                span = sp.empty() ? 1 : (uint32_t)std::strtoul(sp.c_str(), nullptr, 10);
                fstep = st.empty() ? 1 : (uint32_t)std::strtoul(st.c_str(), nullptr, 10);
                fstart = (uint32_t)std::strtoul(s0.c_str(), nullptr, 10);
            } else if (mode == 1) {
                char *e = nullptr;
                const unsigned long p = std::strtoul(l.c_str(), &e, 10);
                const double v = std::strtod(e, nullptr);
                if (p == 0) die("error: bad variableStep position at line " + std::to_string(ln + 1) + "\n");
                add(chrom, p - 1, (uint64_t)p - 1 + span, v);
            } else if (mode == 2) {
                add(chrom, fstart - 1, (uint64_t)fstart - 1 + span, std::strtod(l.c_str(), nullptr));
                fstart += fstep;
            } else {  // bedGraph
                char c[4096];
                unsigned long long s, e;
                double v;
                if (std::sscanf(l.c_str(), "%4095s %llu %llu %lf", c, &s, &e, &v) != 4)
                    die("error: unrecognised line " + std::to_string(ln + 1) + " of " + in + "\n");
                add(c, s, e, v);
            }
        }
        for (const Track &t : tracks) write_bigwig(t, sizes);
    }
    return 0;
}
