// tuning.cpp -- see tuning.hpp.
#include "tuning.hpp"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>

namespace rbamd {

namespace {
int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}
}  // namespace

bool tuning_experimental() {
    static const bool on = env_int("RB_EXPERIMENTAL", 0) != 0;
    return on;
}

namespace {
struct Key {
    const char *name;
    std::atomic<int> Tuning::*field;
    bool experimental;
};
const Key kKeys[] = {
    {"jit", &Tuning::jit, false},
    {"pack", &Tuning::pack, false},
    {"rnea_stream", &Tuning::rnea_stream, false},
    {"single_gpu", &Tuning::single_gpu, false},
    {"fd_form", &Tuning::fd_form, false},
    {"rnea_park", &Tuning::rnea_park, false},
    {"rnea_rev", &Tuning::rnea_rev, false},
    {"grid_factor", &Tuning::grid_factor, true},
    {"rnea_nt", &Tuning::rnea_nt, true},
    {"fd_nt", &Tuning::fd_nt, true},
    {"jit_waves", &Tuning::jit_waves, true},
    {"opaque_consts", &Tuning::opaque_consts, true},
    {"f64_tab", &Tuning::f64_tab, true},
    {"split_rot", &Tuning::split_rot, true},
    {"jit_variant", &Tuning::jit_variant, true},
    {"seq_tail", &Tuning::seq_tail, true},
    {"kin_jit", &Tuning::kin_jit, true},
    {"kin_nt", &Tuning::kin_nt, true},
    {"kernarg_preload", &Tuning::kernarg_preload, true},
};

// RB_<KEY> environment overrides (upper-cased key), experimental ones only with RB_EXPERIMENTAL=1.
void from_env(Tuning &t) {
    for (const Key &k : kKeys) {
        if (k.experimental && !tuning_experimental()) continue;
        std::string var = "RB_";
        for (const char *c = k.name; *c; ++c) var += (char)(*c >= 'a' && *c <= 'z' ? *c - 32 : *c);
        (t.*(k.field)).store(env_int(var.c_str(), (t.*(k.field)).load()));
    }
}
}  // namespace

Tuning &tuning() {
    static Tuning t;
    static const bool init = (from_env(t), true);
    (void)init;
    return t;
}

namespace {
// Sequence count: even when no write is in progress; tuning_set makes it odd, stores, makes it
// even again (writers serialised by g_write).
std::atomic<unsigned> g_generation{2};
std::mutex g_write;
}  // namespace

unsigned tuning_generation() { return g_generation.load(std::memory_order_acquire); }

unsigned tuning_generation_stable() {
    for (;;) {
        const unsigned g = g_generation.load(std::memory_order_acquire);
        if ((g & 1u) == 0) return g;
        std::this_thread::yield();
    }
}

int tuning_set(const char *key, int value) {
    for (const Key &k : kKeys) {
        if (std::strcmp(k.name, key) != 0) continue;
        if (k.experimental && !tuning_experimental()) return 2;
        std::lock_guard<std::mutex> lk(g_write);
        g_generation.fetch_add(1, std::memory_order_acq_rel);
        (tuning().*(k.field)).store(value);
        g_generation.fetch_add(1, std::memory_order_acq_rel);
        return 0;
    }
    return 1;
}

unsigned stream_grid(const void *kfn, int block, unsigned full, int factor) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, unsigned> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return full;
    unsigned resident = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find({dev, kfn});
        if (it != cache.end()) {
            resident = it->second;
        } else {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, block, 0) != hipSuccess || per_cu < 1)
                per_cu = 1;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
                cus = 256;
            resident = (unsigned)per_cu * (unsigned)cus;
            cache[{dev, kfn}] = resident;
        }
    }
    const unsigned g = resident * (unsigned)(factor < 1 ? 1 : factor);
    return g < full ? g : full;
}

}  // namespace rbamd
