// tuning.cpp -- see tuning.hpp.
#include "tuning.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

namespace rbamd {

namespace {
int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}
}  // namespace

Tuning &tuning() {
    static Tuning t = [] {
        Tuning x;
        x.rnea_stream = env_int("RB_RNEA_STREAM", x.rnea_stream);
        x.grid_factor = env_int("RB_GRID_FACTOR", x.grid_factor);
        x.jit = env_int("RB_JIT", x.jit);
        x.rnea_tile = env_int("RB_RNEA_TILE", x.rnea_tile);
        x.rnea_nt = env_int("RB_RNEA_NT", x.rnea_nt);
        x.fd_nt = env_int("RB_FD_NT", x.fd_nt);
        x.opaque_consts = env_int("RB_OPAQUE_CONSTS", x.opaque_consts);
        x.fd_stream = env_int("RB_FD_STREAM", x.fd_stream);
        x.jit_waves = env_int("RB_JIT_WAVES", x.jit_waves);
        x.jit_variant = env_int("RB_JIT_VARIANT", x.jit_variant);
        x.pack = env_int("RB_PACK", x.pack);
        x.f64_tab = env_int("RB_F64_TAB", x.f64_tab);
        x.rnea_seg = env_int("RB_RNEA_SEG", x.rnea_seg);
        x.rnea_tiles = env_int("RB_RNEA_TILES", x.rnea_tiles);
        x.split_rot = env_int("RB_SPLIT_ROT", x.split_rot);
        return x;
    }();
    return t;
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
