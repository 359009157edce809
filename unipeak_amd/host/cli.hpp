// unipeak_amd/host/cli.hpp -- the reference CLIs' flag tables (TCLAP in the
// reference: src/regions.cpp:53-75, src/strand_shift.cpp:52-68,
// src/tags_in_regions.cpp:36-46).  Accepts "-x value", "--long value",
// combined short switches ("-qD"), "--" and trailing positional files;
// parse errors print "error: <msg> for arg <id>" and exit 1 like
// src/regions.cpp:99-101.  --help / --version print and exit 0.
#pragma once

#include <cstdint>

#include <string>
#include <vector>

namespace unipeak {

struct Flag {
    std::string s, l;   // short and long names
    bool is_switch;
    bool required;
    bool seen = false;
    std::string value;
};

class ArgParser {
  public:
    explicit ArgParser(std::vector<Flag> flags) : flags_(std::move(flags)) {}
    void parse(int argc, char **argv);
    const Flag &get(const std::string &s) const;
    bool on(const std::string &s) const { return get(s).seen; }
    std::string str(const std::string &s, const std::string &dflt = "") const;
    double dbl(const std::string &s, double dflt) const;
    uint64_t uint(const std::string &s, uint64_t dflt, uint64_t maxv) const;
    const std::vector<std::string> &files() const { return files_; }

  private:
    [[noreturn]] void fail(const std::string &msg, const std::string &id) const;
    std::vector<Flag> flags_;
    std::vector<std::string> files_;
};

// GPU count for the engine: UNIPEAK_GPUS (0 or unset = every visible device)
int env_gpus();
// the devices the CLIs spread units (tags_in_regions: samples) over: every
// visible HIP device, at most UNIPEAK_GPUS; UNIPEAK_SHARE_DEVICE=N instead
// makes N logical devices that all live on HIP device 0, each with its own
// context (the multi-device path exercised on a one-GPU box)
int cli_device_count();
int cli_physical_device(int logical);

// UNIPEAK_TIMING=1: phase wall times on stderr ("[timing] <phase> <s>"),
// so ingest and the GPU phase can be reported apart
class PhaseTimer {
  public:
    PhaseTimer();
    void mark(const char *phase);  // time since the previous mark
    void accumulate(int slot);     // add the time since the last mark/accumulate to a slot
    void report(int slot, const char *phase) const;
  private:
    bool on_;
    double t_, u_ = 0, s_ = 0, a_last_ = 0, acc_[4] = {0, 0, 0, 0};
};

}  // namespace unipeak
