// unipeak_amd/host/engine.cpp -- see engine.hpp.
#include "engine.hpp"
#include "cli.hpp"

#include <algorithm>
#include <unordered_map>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <mutex>
#include <thread>

namespace unipeak {

// countSum of one add (peakcall.cpp:186-200, quirk Q5): only used here to
// spot head hits; the device recomputes it bit-exactly from the tracks
static double count_sum(const uint32_t *c, size_t S, const std::vector<uint8_t> &control,
                        const std::vector<double> &coeffs) {
    double s = 0;
    if (coeffs.empty()) {
        for (size_t i = 0; i < S; ++i)
            if (!control[i]) s += (double)c[i];
    } else {
        size_t k = 0;
        for (size_t i = 0; i < S && k < coeffs.size(); ++i)
            if (!control[i]) s += (double)c[i] * coeffs[k++];
        for (size_t i = 0; i < S; ++i)
            if (!control[i]) s += (double)c[i];
    }
    return s;
}

namespace {

// one driver-loop iteration (a contig pass): the units it creates and the
// number of add() calls, with add times on a clock local to the iteration
struct IterOut {
    std::vector<UnitBuild> units;
    uint64_t adds = 0;
    bool stepped = false;  // the position loop ran at least once
};

struct MergeSpec {
    size_t S;
    bool directional;
    uint16_t bw;
    const std::vector<uint8_t> *control;
    const std::vector<double> *coeffs;
};

// the position loop of one iteration, src/regions.cpp:311-371 (and
// src/strand_shift.cpp:144-186): every stream whose head lies on this contig
// is consumed position by position; head(i) is stream i's current record,
// advance(i) reads its next one
template <class Head, class Advance>
void merge_iteration(const MergeSpec &m, uint32_t contig, uint32_t lim, uint32_t iteration,
                     uint32_t len, Head head, Advance advance, IterOut &o, uint64_t reserve = 0) {
    const size_t S = m.S;
    std::vector<uint32_t> fh(S), rh(S);
    int cur[2] = {-1, -1};
    auto add = [&](int buffer, int strand, const std::vector<uint32_t> &counts, uint32_t pos) {
        if (cur[buffer] < 0) {
            UnitBuild u;
            u.buffer = buffer;
            u.contig = contig;
            u.len = len;
            u.iteration = iteration;
            if (reserve) {
                const int tr = m.directional ? 0 : strand;
                u.pos[tr].reserve(reserve);
                u.cnt[tr].reserve(reserve * S);
                u.add_pos.reserve(reserve);
                u.add_time.reserve(reserve);
            }
            o.units.push_back(std::move(u));
            cur[buffer] = (int)o.units.size() - 1;
        }
        UnitBuild &u = o.units[cur[buffer]];
        const int track = m.directional ? 0 : strand;
        u.pos[track].push_back(pos);
        for (size_t i = 0; i < S; ++i) u.cnt[track].push_back(counts[i]);
        u.add_pos.push_back(pos);
        u.add_time.push_back(++o.adds);
        if (pos <= m.bw && count_sum(counts.data(), S, *m.control, *m.coeffs) != 0) u.head_hit = true;
    };
    uint32_t pos = 1;
    while (pos <= lim) {
        o.stepped = true;
        bool ff = false, fr = false;
        uint32_t next = lim + 1;
        for (size_t i = 0; i < S; ++i) {
            fh[i] = 0;
            rh[i] = 0;
            const auto *a = &head(i);
            while (a->count != 0 && a->first == pos && a->contig == contig) {
                if (a->forward) { fh[i] += a->count; ff = true; }
                else { rh[i] += a->count; fr = true; }
                a = &advance(i);
            }
            if (a->count != 0 && a->contig == contig && a->first < next) next = a->first;
        }
        if (ff) add(0, 0, fh, pos);
        if (fr) add(m.directional ? 1 : 0, 1, rh, pos);
        pos = next;
    }
    // flushContig(): forward buffer (local time adds+1), then reverse (adds+2)
    for (int b = 0; b < 2; ++b)
        if (cur[b] >= 0) o.units[cur[b]].flush_time = o.adds + 1 + b;
}

// the driver's iteration sequence: contig of iteration i
struct Iterations {
    uint32_t nc;
    bool directional;
    uint32_t count() const { return directional ? 2 * nc : nc; }
    uint32_t contig(uint32_t i) const { return i % nc; }
};

// concatenate iterations on the global event clock: each add ticks once,
// each iteration ends with two flush ticks
void stitch(std::vector<IterOut> &its, PassResult &out) {
    uint64_t base = 0;
    for (IterOut &o : its) {
        for (UnitBuild &u : o.units) {
            for (uint64_t &t : u.add_time) t += base;
            if (u.flush_time) u.flush_time += base;
            out.units.push_back(std::move(u));
        }
        if (o.stepped) out.last_write = base + o.adds;
        base += o.adds + 2;
    }
}

// a stream decoded ahead of the merge: every record read_align() returns
// (the record already read by the caller first), then the count-0 end
using Rec = Tag;

struct Decoded {
    std::unique_ptr<SampleStream> stream;
    std::vector<Rec> recs;
    bool ok = false;
};

void decode_stream(const SampleStream &orig, Decoded &d, unsigned threads) {
    t_defer_errors = true;
    try {
        d.stream = orig.reopen();
        d.stream->expected_tags();
        d.recs.reserve(d.stream->size_hint() + 1);
        const Align *a = &d.stream->read_align();  // the caller's first read
        if (a->count != 0) {
            d.recs.push_back(Rec{a->contig, a->first, a->count, a->forward});
            if (!d.stream->decode_rest(d.recs, threads)) {  // nondirectional: record by record
                for (a = &d.stream->read_align(); a->count != 0; a = &d.stream->read_align())
                    d.recs.push_back(Rec{a->contig, a->first, a->count, a->forward});
            }
        }
        d.recs.push_back(Rec{0, 0, 0, true});
        d.ok = true;
    } catch (const DeferredError &) {
        d.ok = false;
    }
    t_defer_errors = false;
}

}  // namespace

void build_units(std::vector<SampleStream *> &streams, const ContigTable &ct, bool directional,
                 uint16_t bw, const std::vector<uint8_t> &control, const std::vector<double> &coeffs,
                 bool quiet, PassResult &out) {
    (void)quiet;
    const size_t S = streams.size();
    const MergeSpec m{S, directional, bw, &control, &coeffs};
    const Iterations itn{ct.size(), directional};
    const unsigned T = ingest_threads();

    // (1) decode every stream ahead, one thread per stream
    std::vector<Decoded> dec(S);
    const char *ser = std::getenv("UNIPEAK_SERIAL_INGEST");
    bool parallel = !(ser && *ser && *ser != '0');
    if (parallel) {
        std::vector<std::thread> pool;
        std::atomic<size_t> next{0};
        const unsigned outer = (unsigned)std::min<size_t>(T, S), inner = std::max(1u, T / outer);
        for (unsigned t = 0; t < outer; ++t)
            pool.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < S;) decode_stream(*streams[i], dec[i], inner);
            });
        for (auto &th : pool) th.join();
    }
    // (2) which iteration consumes each run of same-contig records: the
    // first one after the previous run's whose contig matches.  A run no
    // iteration reaches leaves its stream stuck there; that case, and any
    // input error, goes to the serial replay below.
    std::vector<std::vector<std::pair<size_t, size_t>>> slice(
        itn.count(), std::vector<std::pair<size_t, size_t>>(S, {0, 0}));
    for (size_t i = 0; i < S && parallel; ++i) {
        const Decoded &d = dec[i];
        if (!d.ok) { parallel = false; break; }
        const size_t n = d.recs.size() - 1;
        int64_t prev = -1;
        for (size_t b = 0; b < n;) {
            const uint32_t c = d.recs[b].contig;
            size_t e = b + 1;
            while (e < n && d.recs[e].contig == c) ++e;
            int64_t it = -1;
            for (uint32_t k = (uint32_t)(prev + 1); k < itn.count(); ++k)
                if (itn.contig(k) == c) { it = k; break; }
            if (it < 0) { parallel = false; break; }
            slice[it][i] = {b, e};
            prev = it;
            b = e;
        }
    }
    std::vector<IterOut> its(itn.count());
    if (parallel) {
        // (3) iterations in parallel, each over its slices of the records
        std::vector<uint32_t> order(itn.count());
        for (uint32_t k = 0; k < itn.count(); ++k) order[k] = k;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
            return ct.length(itn.contig(a)) > ct.length(itn.contig(b));
        });
        std::vector<std::thread> pool;
        std::atomic<size_t> next{0};
        for (unsigned t = 0; t < std::min<size_t>(T, order.size()); ++t)
            pool.emplace_back([&] {
                std::vector<size_t> at(S);
                for (size_t j; (j = next.fetch_add(1)) < order.size();) {
                    const uint32_t k = order[j];
                    for (size_t i = 0; i < S; ++i) at[i] = slice[k][i].first;
                    auto head = [&](size_t i) -> const Rec & {
                        const Decoded &d = dec[i];
                        return at[i] < slice[k][i].second ? d.recs[at[i]] : d.recs.back();
                    };
                    auto advance = [&](size_t i) -> const Rec & {
                        ++at[i];
                        return head(i);
                    };
                    const uint32_t c = itn.contig(k);
                    uint64_t bound = 0;  // adds per buffer are at most the records consumed
                    for (size_t i = 0; i < S; ++i) bound += slice[k][i].second - slice[k][i].first;
                    merge_iteration(m, c, ct.length(c), k, ct.length(c), head, advance, its[k], bound);
                }
            });
        for (auto &th : pool) th.join();
        // the callers' streams continue from where the decode left them (EOF)
        for (size_t i = 0; i < S; ++i) *streams[i] = std::move(*dec[i].stream);
    } else {
        // serial replay on the callers' streams, exactly as the reference reads
        for (uint32_t k = 0; k < itn.count(); ++k) {
            const uint32_t c = itn.contig(k);
            merge_iteration(
                m, c, ct.length(c), k, ct.length(c),
                [&](size_t i) -> const Align & { return streams[i]->last(); },
                [&](size_t i) -> const Align & { return streams[i]->read_align(); }, its[k]);
        }
    }
    dec.clear();
    stitch(its, out);
    out.parallel_ingest = parallel;
}

template <class V>
static uint64_t fnv(const V &v) {
    uint64_t h = 1469598103934665603ull;
    const unsigned char *p = (const unsigned char *)v.data();
    for (size_t i = 0; i < v.size() * sizeof(v[0]); ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

void maybe_dump_units(const PassResult &pr, const std::vector<SampleStream *> &streams) {
    const char *path = std::getenv("UNIPEAK_DUMP_UNITS");
    if (!path || !*path) return;
    FILE *f = std::fopen(path, "w");
    if (!f) fatal(std::string("could not write ") + path);
    std::fprintf(f, "ingest %s\n", pr.parallel_ingest ? "parallel" : "serial");
    std::fprintf(f, "last_write %llu\n", (unsigned long long)pr.last_write);
    for (const UnitBuild &u : pr.units)
        std::fprintf(f, "unit b%d c%u it%u len%u flush%llu head%d n%zu/%zu %016llx %016llx %016llx %016llx %016llx %016llx\n",
                     u.buffer, u.contig, u.iteration, u.len, (unsigned long long)u.flush_time,
                     (int)u.head_hit, u.pos[0].size(), u.pos[1].size(),
                     (unsigned long long)fnv(u.pos[0]), (unsigned long long)fnv(u.pos[1]),
                     (unsigned long long)fnv(u.cnt[0]), (unsigned long long)fnv(u.cnt[1]),
                     (unsigned long long)fnv(u.add_pos), (unsigned long long)fnv(u.add_time));
    for (SampleStream *s : streams)
        std::fprintf(f, "stream %s expected %llu confident %llu oob %llu\n", s->expt_name().c_str(),
                     (unsigned long long)s->expected_tags(), (unsigned long long)s->confident(),
                     (unsigned long long)s->out_of_bounds());
    std::fclose(f);
    exit_now(0);
}

namespace {

struct DeviceJob {
    int dev;
    std::vector<uint32_t> units;  // global unit indices
    up_ctx *ctx = nullptr;
    std::vector<uint32_t> dev_unit;  // device unit id -> global unit index
    std::vector<uint64_t> cand_idx;  // candidate list index of each device region
    int rc = UP_OK;
    std::string err;
};

std::vector<DeviceJob> g_jobs;  // kept alive for shift_scan

void check(int rc, const char *what) {
    if (rc != UP_OK) fatal(std::string(what) + ": " + up_strerror(rc));
}

}  // namespace

// device contexts opened ahead, while the host parses (HIP runtime start-up
// and context creation overlap ingest); run_units takes them over
namespace {
std::thread g_prewarm;
std::vector<up_ctx *> g_pre;
int g_pre_ndev = 0;
}  // namespace

static void join_prewarm() {
    if (g_prewarm.joinable()) g_prewarm.join();
}

void prewarm_devices(int ngpus) {
    g_exit_hook = join_prewarm;  // an input error must not exit mid-initialisation
    (void)ngpus;  // cli_device_count() reads UNIPEAK_GPUS / UNIPEAK_SHARE_DEVICE
    g_prewarm = std::thread([] {
        const int nd = cli_device_count();
        std::vector<up_ctx *> pre(std::max(nd, 0), nullptr);
        for (int d = 0; d < nd; ++d)
            if (up_open(cli_physical_device(d), &pre[d]) != UP_OK) pre[d] = nullptr;
        g_pre = std::move(pre);
        g_pre_ndev = nd;
    });
}

void run_units(const EngineParams &ep, PassResult &out) {
    int ndev = 0;
    if (g_prewarm.joinable()) {
        g_prewarm.join();
        ndev = g_pre_ndev;
    } else {
        ndev = cli_device_count();
    }
    if (ndev < 1) fatal("no HIP device available (the GPU path has no CPU fallback)");
    const size_t S = ep.p.n_samples;
    // Quirk Q1: a unit whose adds all sit at positions <= bw leaves density
    // (and maybe an open region) in its buffer after flushContig(); the
    // library replays such chains, so a chain's units share one device.
    // With a region threshold <= 0 (quirk Q11 live) every unit's last region
    // is still open after its flush and is closed -- relabelled -- in the
    // buffer's next unit (peakcall.cpp:76-78, 164-168), so every unit of a
    // buffer chains to the next one.
    // group[i] = first unit of the chain unit i belongs to.
    std::vector<uint32_t> group(out.units.size());
    {
        const bool q11 = !(ep.p.region_thr > 0);
        int32_t open_prev[2] = {-1, -1};
        for (uint32_t i = 0; i < out.units.size(); ++i) {
            const UnitBuild &u = out.units[i];
            const int b = u.buffer;
            const bool linked = open_prev[b] >= 0;
            group[i] = linked ? group[open_prev[b]] : i;
            const bool in_chain = u.head_hit || linked;
            const bool leaks = !u.add_pos.empty() && u.add_pos.back() <= ep.p.bw;
            open_prev[b] = (q11 || (in_chain && leaks)) ? (int32_t)i : -1;
        }
    }
    // LPT assignment of unit groups to devices by track bytes
    const int nstr = ep.p.nondir ? 2 : 1;
    std::vector<uint64_t> gbytes(out.units.size(), 0);
    for (uint32_t i = 0; i < out.units.size(); ++i)
        gbytes[group[i]] += (uint64_t)out.units[i].len * nstr * S;
    std::vector<uint32_t> order;
    for (uint32_t i = 0; i < out.units.size(); ++i)
        if (group[i] == i) order.push_back(i);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return gbytes[a] > gbytes[b]; });
    std::vector<uint64_t> load(ndev, 0);
    std::vector<int> gdev(out.units.size(), 0);
    g_jobs.assign(ndev, DeviceJob());
    for (int d = 0; d < ndev; ++d) g_jobs[d].dev = d;
    for (uint32_t g : order) {
        int best = 0;
        for (int d = 1; d < ndev; ++d)
            if (load[d] < load[best]) best = d;
        load[best] += gbytes[g];
        gdev[g] = best;
    }
    for (uint32_t i = 0; i < out.units.size(); ++i) g_jobs[gdev[group[i]]].units.push_back(i);
    for (auto &j : g_jobs) std::sort(j.units.begin(), j.units.end());  // buffer order kept

    std::mutex mu;
    auto work = [&](DeviceJob &job) {
        auto fail = [&](int rc, const char *what) {
            job.rc = rc;
            job.err = std::string(what) + ": " + up_strerror(rc);
        };
        if (job.units.empty()) return;
        PhaseTimer tm;
        int rc = UP_OK;
        if (job.dev < (int)g_pre.size() && g_pre[job.dev]) {
            job.ctx = g_pre[job.dev];
            g_pre[job.dev] = nullptr;
        } else if ((rc = up_open(cli_physical_device(job.dev), &job.ctx))) {
            return fail(rc, "up_open");
        }
        tm.mark("  gpu: up_open");
        up_params p = ep.p;
        p.is_control = ep.control.data();
        p.coeffs = ep.coeffs.empty() ? nullptr : ep.coeffs.data();
        p.n_coeffs = (uint32_t)ep.coeffs.size();
        if ((rc = up_set_params(job.ctx, &p))) return fail(rc, "up_set_params");
        if (ep.profile && (rc = up_set_profile_capture(job.ctx, 1))) return fail(rc, "up_set_profile_capture");
        std::vector<uint32_t> tp, tc;
        for (uint32_t gi : job.units) {
            const UnitBuild &u = out.units[gi];
            uint32_t id = 0;
            if ((rc = up_add_unit(job.ctx, u.len, nstr, u.buffer, &id))) return fail(rc, "up_add_unit");
            tm.accumulate(0);
            job.dev_unit.push_back(gi);
            for (int st = 0; st < nstr; ++st) {
                const size_t n = u.pos[st].size();
                if (S == 1) {  // every add of a single sample carries a nonzero count
                    if (n && (rc = up_unit_scatter(job.ctx, id, st, 0, n, u.pos[st].data(), u.cnt[st].data())))
                        return fail(rc, "up_unit_scatter");
                    continue;
                }
                for (size_t s = 0; s < S; ++s) {
                    tp.clear();
                    tc.clear();
                    for (size_t k = 0; k < n; ++k) {
                        const uint32_t c = u.cnt[st][k * S + s];
                        if (c) {
                            tp.push_back(u.pos[st][k]);
                            tc.push_back(c);
                        }
                    }
                    if (!tp.empty() &&
                        (rc = up_unit_scatter(job.ctx, id, st, (uint16_t)s, tp.size(), tp.data(), tc.data())))
                        return fail(rc, "up_unit_scatter");
                }
            }
            if (!u.add_pos.empty()) up_unit_set_last_add(job.ctx, id, u.add_pos.back());
            tm.accumulate(1);
        }
        tm.report(0, "  gpu: up_add_unit");
        tm.report(1, "  gpu: scatter");
        tm.mark("  gpu: units + scatter");
        uint64_t n = 0;
        if ((rc = up_run(job.ctx, &n))) return fail(rc, "up_run");
        tm.mark("  gpu: up_run");
        std::vector<up_region> regs(n);
        std::vector<uint32_t> cnt(n * S);
        if (n && (rc = up_get_regions(job.ctx, regs.data(), cnt.data(), n))) return fail(rc, "up_get_regions");
        tm.mark("  gpu: fetch");
        std::lock_guard<std::mutex> lk(mu);
        for (uint64_t i = 0; i < n; ++i) {
            Candidate c;
            c.r = regs[i];
            c.unit_index = job.dev_unit[regs[i].unit];
            c.counts.assign(cnt.begin() + i * S, cnt.begin() + (i + 1) * S);
            job.cand_idx.push_back(out.cands.size());
            out.cands.push_back(std::move(c));
        }
    };
    std::vector<std::thread> th;
    for (auto &j : g_jobs) th.emplace_back(work, std::ref(j));
    for (auto &t : th) t.join();
    for (auto &j : g_jobs)
        if (j.rc != UP_OK) fatal("GPU device " + std::to_string(j.dev) + ": " + j.err);
}

std::vector<Emitted> order_candidates(const PassResult &out, uint16_t bw, bool accepted_only) {
    std::vector<Emitted> v;
    v.reserve(out.cands.size());
    const uint64_t last_write = out.last_write;
    for (const Candidate &c : out.cands) {
        const UnitBuild &u = out.units[c.unit_index];
        // closed by the first add at pos >= right + bw + 2, else by the flush;
        // regions from the Q1 replay name their closing add (0: the flush);
        // threshold <= 0 (Q11): by the first add past the first add at pos >=
        // right + bw + 1, or (a region left open by the previous unit) past
        // the unit's first add -- an add at the same position (the other
        // strand) retires nothing
        uint64_t key = (uint64_t)c.r.right + bw + 2;
        if (c.r.close_pos == UP_CLOSE_Q11 || c.r.close_pos == UP_CLOSE_Q11_HEAD) {
            auto a1 = u.add_pos.begin();
            if (c.r.close_pos == UP_CLOSE_Q11)
                a1 = std::lower_bound(u.add_pos.begin(), u.add_pos.end(), (uint64_t)c.r.right + bw + 1,
                                      [](uint32_t a, uint64_t k) { return (uint64_t)a < k; });
            key = a1 != u.add_pos.end() ? (uint64_t)*a1 + 1 : ~0ull;
        } else if (c.r.close_pos != UP_CLOSE_RULE) {
            key = c.r.close_pos ? c.r.close_pos : ~0ull;
        }
        auto it = std::lower_bound(u.add_pos.begin(), u.add_pos.end(), key,
                                   [](uint32_t a, uint64_t k) { return (uint64_t)a < k; });
        const uint64_t t = it != u.add_pos.end() ? u.add_time[it - u.add_pos.begin()] : u.flush_time;
        v.push_back(Emitted{&c, t, false, u.buffer == 0});
    }
    std::stable_sort(v.begin(), v.end(), [](const Emitted &a, const Emitted &b) {
        if (a.close_time != b.close_time) return a.close_time < b.close_time;
        return a.c->r.left < b.c->r.left;
    });
    // Q2: the reverse buffer's first candidate keeps the ctor's forward label
    for (Emitted &e : v)
        if (out.units[e.c->unit_index].buffer == 1) {
            e.forward_label = true;
            break;
        }
    for (Emitted &e : v) e.written = e.c->r.accepted && e.close_time <= last_write;  // Q3
    if (accepted_only) {
        std::vector<Emitted> a;
        for (const Emitted &e : v)
            if (e.c->r.accepted) a.push_back(e);
        return a;
    }
    return v;
}

// per device: the positions of `regs` it holds (its local candidate
// indices); one hash of the device's candidate list instead of a search per
// region
static void device_regions(const PassResult &out, const DeviceJob &job,
                           const std::vector<const Candidate *> &regs, std::vector<uint64_t> &idx,
                           std::vector<size_t> &where) {
    std::unordered_map<uint64_t, uint64_t> local;
    local.reserve(job.cand_idx.size() * 2);
    for (size_t i = 0; i < job.cand_idx.size(); ++i) local.emplace(job.cand_idx[i], (uint64_t)i);
    idx.clear();
    where.clear();
    for (size_t k = 0; k < regs.size(); ++k) {
        auto it = local.find((uint64_t)(regs[k] - out.cands.data()));
        if (it == local.end()) continue;
        idx.push_back(it->second);
        where.push_back(k);
    }
}

void shift_scan(const EngineParams &ep, PassResult &out, const std::vector<const Candidate *> &regs,
                uint16_t max_shift, std::vector<double> &table) {
    (void)ep;
    const size_t W = (size_t)max_shift + 1;
    table.assign(regs.size() * W, 0.0);
    std::vector<uint64_t> idx;
    std::vector<size_t> where;
    for (DeviceJob &job : g_jobs) {
        if (!job.ctx) continue;
        device_regions(out, job, regs, idx, where);
        if (idx.empty()) continue;
        std::vector<double> t(idx.size() * W);
        check(up_shift_scan(job.ctx, idx.data(), idx.size(), max_shift, t.data()), "up_shift_scan");
        for (size_t j = 0; j < idx.size(); ++j)
            std::copy(t.begin() + j * W, t.begin() + (j + 1) * W, table.begin() + where[j] * W);
    }
}

void shift_best(const EngineParams &ep, PassResult &out, const std::vector<const Candidate *> &regs,
                uint16_t max_shift, std::vector<uint16_t> &best, std::vector<double> &best_corr) {
    (void)ep;
    best.assign(regs.size(), 0);
    best_corr.assign(regs.size(), -1.0);
    std::vector<uint64_t> idx;
    std::vector<size_t> where;
    for (DeviceJob &job : g_jobs) {
        if (!job.ctx) continue;
        device_regions(out, job, regs, idx, where);
        if (idx.empty()) continue;
        std::vector<uint16_t> b(idx.size());
        std::vector<double> c(idx.size());
        check(up_shift_best(job.ctx, idx.data(), idx.size(), max_shift, b.data(), c.data()), "up_shift_best");
        for (size_t j = 0; j < idx.size(); ++j) {
            best[where[j]] = b[j];
            best_corr[where[j]] = c[j];
        }
    }
}

void ProfileSink::header() {  // FormatOutStream::trackHeader, format.cpp:1164-1219
    std::fprintf(fp, "track name=\"%s", name.c_str());
    if (directional) std::fputs(forward ? " +" : " -", fp);
    std::fputc('"', fp);
    if (directional) std::fprintf(fp, " description=\"%s\"", forward ? name.c_str() : " ");
    std::fputs(" priority=2 visibility=", fp);  // PROFILE_PRIORITY, defaults.hpp:42
    if (directional)
        std::fputs(forward ? "full type=wiggle_0 alwaysZero=on color=0,0,255"
                           : "full type=wiggle_0 alwaysZero=on color=255,0,0 altColor=255,0,0", fp);
    else
        std::fputs("full type=wiggle_0 alwaysZero=on color=191,0,191", fp);
    if (!assembly.empty()) std::fprintf(fp, " db=%s", assembly.c_str());
    std::fputc('\n', fp);
}

void ProfileSink::write(bool fwd, uint32_t c, uint64_t pos, double score) {
    if (score == 0) return;  // format.cpp:1092
    if (directional) {
        if (!have_contig || forward != fwd) {
            forward = fwd;
            have_contig = false;
            header();
        }
    } else if (!have_contig) {
        header();
    }
    if (!have_contig || contig != c) {
        contig = c;
        have_contig = true;
        std::fprintf(fp, "variableStep chrom=%s\n", ct->name(c).c_str());
    }
    // ostream << double: 6 significant digits (%g); reverse strand negated
    std::fprintf(fp, (directional && !fwd) ? "%llu -%g\n" : "%llu %g\n", (unsigned long long)pos, score);
}

void write_profile(const PassResult &pr, uint16_t bw, ProfileSink &sink) {
    // device context and unit id of every global unit
    std::vector<std::pair<up_ctx *, uint32_t>> where(pr.units.size(), {nullptr, 0});
    for (const DeviceJob &j : g_jobs)
        for (size_t k = 0; k < j.dev_unit.size(); ++k) where[j.dev_unit[k]] = {j.ctx, (uint32_t)k};
    // Units the exact replay produced (quirk Q1 heads, -r <= 0, bw > 255)
    // hand over their retirements as the state machine wrote them: every
    // nonzero (pos, score) with the add() -- or flush -- whose retirement loop
    // wrote it.  Positions at or after a resync point follow the dense KDE.
    struct Replayed { uint32_t resync = 0; std::vector<uint32_t> event, pos; std::vector<double> score; };
    std::vector<Replayed> rep(pr.units.size());
    for (uint32_t k = 0; k < pr.units.size(); ++k) {
        Replayed &r = rep[k];
        uint64_t n = 0;
        int rc = up_unit_replay_profile(where[k].first, where[k].second, &r.resync, &n, nullptr, nullptr,
                                        nullptr, 0);
        if (rc != UP_OK) fatal(std::string("up_unit_replay_profile: ") + up_strerror(rc));
        r.event.resize(n);
        r.pos.resize(n);
        r.score.resize(n);
        if (n && (rc = up_unit_replay_profile(where[k].first, where[k].second, &r.resync, &n, r.event.data(),
                                              r.pos.data(), r.score.data(), n)) != UP_OK)
            fatal(std::string("up_unit_replay_profile: ") + up_strerror(rc));
    }
    // retirement events in the driver's call order: add() at p after q retires
    // q-bw .. q-bw+min(W,p-q)-1 (peakcall.cpp:171-184); flushContig()
    // retires q-bw .. q+bw.  A replayed unit's entries go out at the event
    // that wrote them, before the dense positions of the same event.
    struct Ev { uint64_t t; uint32_t unit; int kind; int64_t lo, hi; };  // kind 0: replayed [lo, hi) entries
    std::vector<Ev> ev;
    const int64_t W = 2 * (int64_t)bw + 1;
    for (uint32_t k = 0; k < pr.units.size(); ++k) {
        const UnitBuild &u = pr.units[k];
        const Replayed &r = rep[k];
        for (size_t i = 0; i < r.event.size();) {  // runs of one event
            size_t j = i;
            while (j < r.event.size() && r.event[j] == r.event[i]) ++j;
            const uint32_t e = r.event[i];
            uint64_t t;
            if (e == UP_FLUSH_EVENT) t = u.flush_time;
            else if (e < u.add_time.size()) t = u.add_time[e];
            else fatal("-w: the replay's add index exceeds the unit's adds");
            ev.push_back({t, k, 0, (int64_t)i, (int64_t)j});
            i = j;
        }
        if (r.resync == UP_FLUSH_EVENT) continue;  // replayed to the end
        const int64_t x0 = r.resync ? (int64_t)r.resync : 1;  // dense from the resync point on
        int64_t q = 0;
        for (size_t i = 0; i < u.add_pos.size(); ++i) {
            const int64_t p = u.add_pos[i];
            if (q != 0 && p > q) {
                const int64_t n = std::min<int64_t>(W, p - q);
                const int64_t lo = std::max<int64_t>({1, q - bw, x0}), hi = q - bw + n - 1;
                if (lo <= hi) ev.push_back({u.add_time[i], k, 1, lo, hi});
            }
            q = p;
        }
        if (q != 0) {
            const int64_t lo = std::max<int64_t>({1, q - bw, x0}), hi = q + bw;
            if (lo <= hi) ev.push_back({u.flush_time, k, 1, lo, hi});
        }
    }
    std::stable_sort(ev.begin(), ev.end(), [](const Ev &a, const Ev &b) {
        return a.t != b.t ? a.t < b.t : a.kind < b.kind;
    });
    // per-unit cache of one chunk of the device profile
    constexpr uint32_t kChunkPos = 1u << 22;
    struct Cache { int64_t first = -1; std::vector<double> f, r; };
    std::vector<Cache> cache(pr.units.size());
    for (const Ev &e : ev) {
        const UnitBuild &u = pr.units[e.unit];
        if (e.kind == 0) {
            const Replayed &r = rep[e.unit];
            for (int64_t i = e.lo; i < e.hi; ++i) sink.write(u.buffer == 0, u.contig, r.pos[i], r.score[i]);
            continue;
        }
        Cache &c = cache[e.unit];
        for (int64_t x = e.lo; x <= e.hi; ++x) {
            if (c.first < 0 || x < c.first || x >= c.first + (int64_t)kChunkPos) {
                c.first = ((x - 1) / kChunkPos) * kChunkPos + 1;
                const uint64_t dom_end = (uint64_t)u.len + bw;  // highest position a flush retires
                const uint32_t n = (uint32_t)std::min<uint64_t>(kChunkPos, dom_end - (uint64_t)c.first + 1);
                c.f.assign(n, 0.0);
                c.r.assign(n, 0.0);
                const int rc = up_unit_profile_range(where[e.unit].first, where[e.unit].second,
                                                     (uint64_t)c.first, n, c.f.data(), c.r.data());
                if (rc != UP_OK) fatal(std::string("up_unit_profile_range: ") + up_strerror(rc));
            }
            const size_t i = (size_t)(x - c.first);
            if (i >= c.f.size()) continue;  // beyond the scan domain: never scored
            sink.write(u.buffer == 0, u.contig, (uint64_t)x, c.f[i] + c.r[i]);
        }
    }
}

void release_devices() {
    join_prewarm();
    for (DeviceJob &j : g_jobs)
        if (j.ctx) up_close(j.ctx);
    g_jobs.clear();
    for (up_ctx *c : g_pre)
        if (c) up_close(c);
    g_pre.clear();
}

}  // namespace unipeak
