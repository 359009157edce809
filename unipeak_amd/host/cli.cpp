// unipeak_amd/host/cli.cpp -- see cli.hpp.
#include "cli.hpp"

#include <cstdio>
#include <ctime>
#include <sys/resource.h>

#include <cstdlib>
#include <iostream>

#include "wigio.hpp"
#include "unipeak_hip.h"

namespace unipeak {

void ArgParser::fail(const std::string &msg, const std::string &id) const {
    std::cerr << "error: " << msg << " for arg " << id << std::endl << std::endl;
    std::exit(1);
}

void ArgParser::parse(int argc, char **argv) {
    bool only_files = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (!only_files && a == "--") { only_files = true; continue; }
        if (!only_files && (a == "--version" || a == "-v")) {
            std::cout << std::endl << argv[0] << "  version: 1.0" << std::endl << std::endl;
            std::exit(0);
        }
        if (!only_files && (a == "--help" || a == "-h")) {
            std::cout << "See README.TXT for more information" << std::endl;
            std::exit(0);
        }
        if (only_files || a.size() < 2 || a[0] != '-') {
            files_.push_back(a);
            continue;
        }
        Flag *hit = nullptr;
        for (Flag &f : flags_)
            if ((a[1] != '-' && a.substr(1) == f.s) || (a[1] == '-' && !f.l.empty() && a.substr(2) == f.l))
                hit = &f;
        if (hit) {
            if (hit->seen) fail("Argument already set!", "-" + hit->s + " (--" + hit->l + ")");
            hit->seen = true;
            if (!hit->is_switch) {
                if (i + 1 >= argc) fail("Missing a value for this argument!", "-" + hit->s + " (--" + hit->l + ")");
                hit->value = argv[++i];
            }
            continue;
        }
        // combined short switches
        bool all = a[1] != '-';
        for (size_t k = 1; all && k < a.size(); ++k) {
            bool found = false;
            for (Flag &f : flags_)
                if (f.is_switch && f.s.size() == 1 && f.s[0] == a[k]) found = true;
            all = found;
        }
        if (!all) fail("Couldn't find match for argument", a);
        for (size_t k = 1; k < a.size(); ++k)
            for (Flag &f : flags_)
                if (f.is_switch && f.s.size() == 1 && f.s[0] == a[k]) f.seen = true;
    }
    for (const Flag &f : flags_)
        if (f.required && !f.seen) fail("Required argument missing", "-" + f.s + " (--" + f.l + ")");
}

const Flag &ArgParser::get(const std::string &s) const {
    for (const Flag &f : flags_)
        if (f.s == s) return f;
    std::cerr << "internal: unknown flag " << s << std::endl;
    std::abort();
}

std::string ArgParser::str(const std::string &s, const std::string &dflt) const {
    const Flag &f = get(s);
    return f.seen ? f.value : dflt;
}

double ArgParser::dbl(const std::string &s, double dflt) const {
    const Flag &f = get(s);
    if (!f.seen) return dflt;
    double v;
    if (!lex_double(f.value, &v))
        fail("Couldn't read argument value from string '" + f.value + "'", "-" + f.s + " (--" + f.l + ")");
    return v;
}

uint64_t ArgParser::uint(const std::string &s, uint64_t dflt, uint64_t maxv) const {
    const Flag &f = get(s);
    if (!f.seen) return dflt;
    uint64_t v;
    if (!lex_uint(f.value, maxv, &v))
        fail("Couldn't read argument value from string '" + f.value + "'", "-" + f.s + " (--" + f.l + ")");
    return v;
}

static double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void cpu_s(double *user, double *sys);

PhaseTimer::PhaseTimer() : on_(false), t_(now_s()) {
    cpu_s(&u_, &s_);
    const char *e = std::getenv("UNIPEAK_TIMING");
    on_ = e && *e && *e != '0';
}

static void cpu_s(double *user, double *sys) {
    rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    *user = (double)ru.ru_utime.tv_sec + 1e-6 * (double)ru.ru_utime.tv_usec;
    *sys = (double)ru.ru_stime.tv_sec + 1e-6 * (double)ru.ru_stime.tv_usec;
}

void PhaseTimer::mark(const char *phase) {
    const double t = now_s();
    double u, s;
    cpu_s(&u, &s);
    if (on_)
        std::fprintf(stderr, "[timing] %s %.3f s (cpu user %.3f sys %.3f)\n", phase, t - t_, u - u_, s - s_);
    t_ = t;
    u_ = u;
    s_ = s;
    a_last_ = t;
}

void PhaseTimer::accumulate(int slot) {
    const double t = now_s();
    if (a_last_ == 0) a_last_ = t_;
    acc_[slot] += t - a_last_;
    a_last_ = t;
}

void PhaseTimer::report(int slot, const char *phase) const {
    if (on_) std::fprintf(stderr, "[timing] %s %.3f s\n", phase, acc_[slot]);
}

int env_gpus() {
    const char *e = std::getenv("UNIPEAK_GPUS");
    return e ? std::atoi(e) : 0;
}

static int env_share() {
    const char *e = std::getenv("UNIPEAK_SHARE_DEVICE");
    return e ? std::atoi(e) : 0;
}

int cli_device_count() {
    int nd = 0;
    up_device_count(&nd);
    if (nd < 1) return nd;
    if (env_share() > 0) return env_share();
    const int g = env_gpus();
    return g > 0 && g < nd ? g : nd;
}

int cli_physical_device(int d) { return env_share() > 0 ? 0 : d; }

}  // namespace unipeak
