// unipeak_amd/host/engine.hpp -- host orchestration of the hot path.
//
// The reference drives two ProfileBuffers position by position while
// merging S sorted wiggle streams (src/regions.cpp:309-391,
// src/strand_shift.cpp:143-190).  Here the same merge is replayed once on
// the host over the parsed streams to build, for every (buffer, contig
// pass) "unit", the dense count tracks the GPU scans and the event clock
// that fixes when each region is closed and written (quirks Q2-Q4).  The
// units then run on one or more MI355X through the C-ABI, and the candidate
// regions come back for emission in the reference's order.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "unipeak_hip.h"
#include "wigio.hpp"

namespace unipeak {

struct UnitBuild {
    int buffer = 0;          // 0: forward ProfileBuffer, 1: reverse ProfileBuffer
    uint32_t contig = 0;
    uint32_t len = 0;        // contig length
    uint32_t iteration = 0;  // driver loop iteration (contig pass) that fed it
    // per strand (0 forward adds, 1 reverse adds): positions and [n][S] counts
    std::vector<uint32_t> pos[2];
    std::vector<uint32_t> cnt[2];
    // every add() this buffer received in this pass, in call order
    std::vector<uint32_t> add_pos;
    std::vector<uint64_t> add_time;
    uint64_t flush_time = 0;
    bool head_hit = false;   // an add with countSum != 0 at pos <= bw (quirk Q1)
};

struct Candidate {
    up_region r;             // from the device
    std::vector<uint32_t> counts;  // exptSums, S entries
    uint32_t unit_index = 0; // into the UnitBuild list
};

struct PassResult {
    std::vector<UnitBuild> units;
    uint64_t last_write = 0;            // event clock after the last loop step (Q3)
    bool parallel_ingest = false;       // built by the per-iteration parallel merge
    std::vector<Candidate> cands;       // all candidates, any order
};

struct EngineParams {
    up_params p{};
    std::vector<uint8_t> control;
    std::vector<double> coeffs;
    int ngpus = 0;           // 0: all visible devices
    bool profile = false;    // -w: capture the exact replay's retirements too
};

// replay the merge loop; directional = two buffers and two passes
// (regions), otherwise one buffer (regions -D, strand_shift)
void build_units(std::vector<SampleStream *> &streams, const ContigTable &ct,
                 bool directional, uint16_t bw, const std::vector<uint8_t> &control,
                 const std::vector<double> &coeffs, bool quiet, PassResult &out);

// UNIPEAK_DUMP_UNITS=<file>: write a digest of the merge result (units, add
// clocks, stream counters) and exit before the GPU phase -- lets CPU tests
// check the parallel ingest against the serial replay (UNIPEAK_SERIAL_INGEST=1)
void maybe_dump_units(const PassResult &pr, const std::vector<SampleStream *> &streams);

// start the HIP runtime and open the device contexts on a helper thread
// (overlaps ingest); optional, run_units opens them itself otherwise
void prewarm_devices(int ngpus);

// run every unit on the GPU(s); fills out.cands
void run_units(const EngineParams &ep, PassResult &out);

// candidates in closing-event order; sets *written for those the reference
// writes (Q3) and *fwd_label for the printed orientation (Q2)
struct Emitted {
    const Candidate *c;
    uint64_t close_time;
    bool written;
    bool forward_label;
};
std::vector<Emitted> order_candidates(const PassResult &out, uint16_t bw, bool accepted_only);

// strandCorr(shift) table for accepted candidates (strand_shift), on GPU
void shift_scan(const EngineParams &ep, PassResult &out, const std::vector<const Candidate *> &regs,
                uint16_t max_shift, std::vector<double> &table);
// strand_shift's per-region choice from the same table, reduced on the GPU
// (up_shift_best): first shift of the largest correlation above -1
void shift_best(const EngineParams &ep, PassResult &out, const std::vector<const Candidate *> &regs,
                uint16_t max_shift, std::vector<uint16_t> &best, std::vector<double> &best_corr);

// -w density profile (regions.cpp:276-284): every processed position with a
// nonzero score, written when the reference's processPosition writes it --
// at the add() (or flush) that retires it, interleaved across the two
// buffers by the replayed event clock (misc/format.cpp:1091-1132)
struct ProfileSink {
    std::FILE *fp = nullptr;
    const ContigTable *ct = nullptr;
    bool directional = true;
    std::string name, assembly;
    bool have_contig = false, forward = true;
    uint32_t contig = 0;
    void header();
    void write(bool fwd, uint32_t contig, uint64_t pos, double score);
};
void write_profile(const PassResult &pr, uint16_t bw, ProfileSink &sink);

void release_devices();

}  // namespace unipeak
