// capi.cpp -- the extern "C" boundary (include/rigidbody.h, include/rigidbody_batch.h).
//
// Drop-in for the Rust cdylib rigidbody_bindings (rigidbody_bindings/src/lib.rs:8-78):
// same six symbols and result layouts, plus batched device-pointer entry points.
// Every batched entry point runs a HIP kernel on the current device (no CPU fallback).  The
// reference's single-configuration queries run on the calling host thread with the same
// lane bodies compiled for the host (host_eval.cpp: SURVEY §8(d) config 1 is a CPU path, and
// a GPU round trip costs ~25x the recursion), unless the model needs hipRTC (trees) or the
// caller asks for the GPU (tuning single_gpu).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rigidbody_batch.h"
#include "kernels.hpp"
#include "model.hpp"
#include "tuning.hpp"
#include "jit.hpp"
#include "host_eval.hpp"

#include "fr3_embedded.inc"  // kFr3Urdf: compact FR3 description (tools/gen_fixtures.py)

#define RB_VERSION "rigidbody-rs_amd 0.2.0 (gfx950)"

static const char *const kKindMsg = "kind must be 0 rnea, 1 fd, 2 crba, 3 rollout, 4 fwd_kin, 5 jac or 6 rnea_fd";

namespace {

thread_local std::string g_last_error;
// Why a launcher refused (a tree model without its hipRTC kernel); hip_err reports it.
thread_local std::string t_launch_note;

int set_err(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

int hip_err(hipError_t e, const char *where) {
    std::string msg = std::string(where) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
    if (!t_launch_note.empty()) {
        msg += ": " + t_launch_note;
        t_launch_note.clear();
        return set_err(RB_ERR_UNSUPPORTED, msg);
    }
    return set_err(RB_ERR_HIP, msg);
}

bool env_flag(const char *name, bool dflt) {
    const char *v = std::getenv(name);
    if (!v || !*v) return dflt;
    return !(v[0] == '0' || v[0] == 'n' || v[0] == 'N' || v[0] == 'f' || v[0] == 'F');
}

// fp32 kernels use the hardware sin/cos (v_sin_f32 / v_cos_f32) unless RB_FAST_TRIG=0.
bool fast_trig() {
    static const bool fast = env_flag("RB_FAST_TRIG", true);
    return fast;
}

struct DeviceConsts {
    float *f32 = nullptr;
    double *f64 = nullptr;
};

}  // namespace

struct Multibody {
    rbamd::Model model;
    std::vector<float> pk32;
    std::vector<double> pk64;
    mutable std::mutex mu;
    mutable std::map<int, DeviceConsts> dev;
    // model-specialised hipRTC kernels, keyed by (device, kind, dtype, trig, tuning tag, form)
    mutable std::map<std::string, rbamd::JitKernel> jit;
    mutable std::map<std::string, int> jit_device;
    // per-launch fast path of jit_get: [device][kind][f64][fast trig][requested pack][tail] ->
    // the kernel resolved under one tuning generation, published as ONE pointer to a record
    // {generation, kernel}.  There is one record per (slot, kernel) pair, so the records are
    // bounded by slots x kernels however often the tuning changes: a record's kernel never
    // changes, its generation is re-stamped only when ITS slot resolves to that kernel again,
    // and records live in jit_pub (std::map nodes never move) until free.  A reader that sees
    // the current generation in the record its slot points at has that slot's kernel.
    struct JitPub {
        std::atomic<unsigned> gen{0};
        const rbamd::JitKernel *jk = nullptr;
    };
    mutable std::map<std::pair<const void *, const rbamd::JitKernel *>, JitPub> jit_pub;
    mutable std::atomic<const JitPub *> jit_fast[16][rbamd::kJitKinds][2][2][6][4] = {};  // last: tail > 0, nt override
    // device_consts fast path: the uploaded constant blocks per device (set once, never moved)
    mutable std::atomic<const void *> dc_fast[16][2] = {};
};

namespace {

constexpr int kMaxTreeDof = 64;

Multibody *make(rbamd::Model &&m) {
    if (!m.axes_supported()) {
        set_err(RB_ERR_UNSUPPORTED,
                "non-z joint axis: the reference injects joint motion about local z "
                "(multibody.rs:130-138,144); pass RB_MODEL_GENERAL_AXES for general axes");
        return nullptr;
    }
    // The reference's serial revolute chains run on the precompiled kernels (dofs.hpp) or
    // their model-specialised versions; trees and prismatic joints only on the latter, which
    // exist for any DOF count.
    if (m.serial_revolute() ? !rbamd::dof_supported(m.n) : m.n > kMaxTreeDof) {
        set_err(RB_ERR_DOF, m.serial_revolute() ? "no kernel compiled for " + std::to_string(m.n) + " DOF"
                                                : "tree models support at most 64 DOF, got " + std::to_string(m.n));
        return nullptr;
    }
    Multibody *mb = new Multibody();
    mb->pk32 = m.pack_f32();
    mb->pk64 = m.pack_f64();
    mb->model = std::move(m);
    return mb;
}

// Device copy of the packed model constants on the current device (uploaded once).
template <typename T>
int device_consts(const Multibody *mb, const T **out) {
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return hip_err(e, "hipGetDevice");
    std::atomic<const void *> *fastp = (d >= 0 && d < 16) ? &mb->dc_fast[d][sizeof(T) == 8 ? 1 : 0] : nullptr;
    if (fastp) {
        if (const void *p = fastp->load(std::memory_order_acquire)) {
            *out = static_cast<const T *>(p);
            return RB_OK;
        }
    }
    std::lock_guard<std::mutex> lk(mb->mu);
    DeviceConsts &dc = mb->dev[d];
    if constexpr (sizeof(T) == 4) {
        if (!dc.f32) {
            void *p = nullptr;
            size_t bytes = mb->pk32.size() * sizeof(float);
            if ((e = hipMalloc(&p, bytes)) != hipSuccess) return hip_err(e, "hipMalloc(model)");
            if ((e = hipMemcpy(p, mb->pk32.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess) {
                (void)hipFree(p);
                return hip_err(e, "hipMemcpy(model)");
            }
            dc.f32 = static_cast<float *>(p);
        }
        *out = reinterpret_cast<const T *>(dc.f32);
        if (fastp) fastp->store(dc.f32, std::memory_order_release);
    } else {
        if (!dc.f64) {
            void *p = nullptr;
            size_t bytes = mb->pk64.size() * sizeof(double);
            if ((e = hipMalloc(&p, bytes)) != hipSuccess) return hip_err(e, "hipMalloc(model)");
            if ((e = hipMemcpy(p, mb->pk64.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess) {
                (void)hipFree(p);
                return hip_err(e, "hipMemcpy(model)");
            }
            dc.f64 = static_cast<double *>(p);
        }
        *out = reinterpret_cast<const T *>(dc.f64);
        if (fastp) fastp->store(dc.f64, std::memory_order_release);
    }
    return RB_OK;
}

// The hipRTC kernel of `kind` for this model on the current device, or nullptr (the
// precompiled generic kernel then runs).
// pack: configurations per lane, 0 = the jit_pack policy (jit.cpp).
// tail: percent of a sequential-pair RNEA launch run one per lane (jit_seq_tail); other kinds 0.
const rbamd::JitKernel *jit_get(const Multibody *mb, rbamd::JitKind kind, bool f64, bool fast, int pack = 0,
                                int tail = 0, int nt = -1) {
    if (!rbamd::jit_enabled()) return nullptr;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return nullptr;
    const bool fst = fast && !f64;
    std::atomic<const Multibody::JitPub *> *slot = nullptr;
    if (d >= 0 && d < 16 && (int)kind >= 0 && (int)kind < rbamd::kJitKinds && pack >= 0 && pack < 6) {
        slot = &mb->jit_fast[d][(int)kind][f64 ? 1 : 0][fst ? 1 : 0][pack][(tail > 0 ? 1 : 0) | (nt >= 0 ? 2 : 0)];
        if (const Multibody::JitPub *p = slot->load(std::memory_order_acquire))
            if (p->gen.load(std::memory_order_acquire) == rbamd::tuning_generation()) return p->jk;
    }
    const int pack_req = pack;
    std::lock_guard<std::mutex> lk(mb->mu);
    // The tuning generation is a sequence count (tuning.cpp): odd while rb_set_tuning writes,
    // bumped again after.  The key and the kernel source both read the tuning knobs, so they are
    // resolved between two reads of one even generation; a write in between resolves again (a
    // kernel built from a mix of two tunings is never stored under either key).
    for (;;) {
        const unsigned gen = rbamd::tuning_generation_stable();
        int pk = pack_req > 0 ? pack_req : rbamd::jit_model_pack(mb->model, kind, f64, 0);
        const int tl = (kind == rbamd::JitKind::Rnea && pk == 3) ? tail : 0;
        const std::string key = std::to_string(d) + ":k" + std::to_string((int)kind) + (f64 ? ":f64" : ":f32") +
                                (fst ? ":fast" : ":precise") + rbamd::jit_tag(kind, f64, mb->model.n) + ":q" +
                                std::to_string(pk) + ":st" + std::to_string(tl) + ":n" + std::to_string(nt);
        auto it = mb->jit.find(key);
        if (it == mb->jit.end()) {
            rbamd::JitKernel built = rbamd::jit_build(mb->model, kind, f64, fst, pk, tl, nt);
            if (rbamd::tuning_generation() != gen) {  // the tuning moved under the build
                if (built.module) (void)hipModuleUnload(built.module);
                continue;
            }
            it = mb->jit.emplace(key, std::move(built)).first;
            mb->jit_device[key] = d;
        }
        const rbamd::JitKernel *res = it->second.function ? &it->second : nullptr;
        if (rbamd::tuning_generation() != gen) continue;
        if (slot && res) {
            // jk is written once, when the record is created (the key holds the same pointer), and
            // never again: fast-path readers may hold the record while this re-stamps gen
            auto ins = mb->jit_pub.try_emplace({(const void *)slot, res});
            Multibody::JitPub &rec = ins.first->second;
            if (ins.second) rec.jk = res;
            rec.gen.store(gen, std::memory_order_release);
            slot->store(&rec, std::memory_order_release);
        }
        return res;
    }
}

// Smallest batch for which the auto policy takes the sequential-pair fp64 RNEA (jit_pack 3):
// it halves the waves, so below two resident rounds of the one-per-lane kernel (4 waves/SIMD x
// 1024 SIMDs x 64 lanes x 2) the one-per-lane kernel keeps more of the chip busy.
constexpr uint32_t kSeqMinBatch = 1u << 19;

// The hipRTC kernel variant a launch takes: configurations per lane (0 = the jit_pack policy),
// the sequential pair's one-per-lane tail, the non-temporal override and the fp32 trig form.
// The launch paths and the inspection entry points (multibody_jit_source_ex) share it.
struct JitShape {
    int pack = 0, tail = 0, nt = -1;
    bool fast = false;
};
JitShape jit_shape(const Multibody *mb, rbamd::JitKind kind, bool f64, uint32_t B, bool tiled);

const rbamd::JitKernel *jit_shaped(const Multibody *mb, rbamd::JitKind kind, bool f64, uint32_t B, bool tiled) {
    const JitShape sh = jit_shape(mb, kind, f64, B, tiled);
    return jit_get(mb, kind, f64, sh.fast, sh.pack, sh.tail, sh.nt);
}

JitShape rnea_shape(const Multibody *mb, bool f64, uint32_t B, bool tiled) {
    // fp32 chains up to 8 links on the tiled layout at large batches: the sequential pair too
    // (FR3 2^20 22.0-22.1 vs 22.3-24.0 us on two boxes, profiles/r04/ab/ab_r32_seq*.log), with
    // ordinary (temporal) loads and stores (tuning.hpp rnea_nt; the 30-link chain and the 14-DOF
    // tree keep nt = 3)
    const bool big32 = !f64 && tiled && B >= kSeqMinBatch && mb->model.n <= 8;
    JitShape sh;
    sh.pack = rbamd::tuning().pack >= 0 ? 0 : big32 ? 3 : B < kSeqMinBatch ? 1 : 0;
    sh.nt = (big32 && rbamd::tuning().rnea_nt < 0) ? 0 : -1;
    sh.tail = rbamd::jit_seq_tail(tiled);
    return sh;
}

const rbamd::JitKernel *jit_rnea(const Multibody *mb, bool f64, uint32_t B, bool tiled) {
    return jit_shaped(mb, rbamd::JitKind::Rnea, f64, B, tiled);
}

// A tree / prismatic model has no precompiled kernel: without its hipRTC kernel the launch
// is refused (hipErrorNotSupported, reported as RB_ERR_UNSUPPORTED with the reason).
hipError_t no_generic(const Multibody *mb) {
    std::string why = "kinematic-tree / prismatic models run only on model-specialised (hipRTC) kernels";
    if (!rbamd::jit_enabled()) {
        why += ", which are disabled (RB_JIT=0 / rb_set_tuning(\"jit\", 0))";
    } else {
        std::lock_guard<std::mutex> lk(mb->mu);
        for (auto &kv : mb->jit)
            if (!kv.second.error.empty()) why += "; hipRTC: " + kv.second.error.substr(0, 400);
    }
    t_launch_note = why;
    return hipErrorNotSupported;
}

// Smallest batch for which the auto policy takes the paired-lane kernel: one resident round
// of it (2 blocks of 512 configurations per CU x 256 CUs) -- 2^18.
constexpr uint32_t kPackMinBatch = 1u << 18;
// fp32 mass-matrix forward dynamics at small batches: one wave per SIMD at most, so the launch
// time follows each wave's instruction stream; the wave splits (fdh_body.hip.hpp) halve it.
// Up to 2^17 configurations the one-per-lane split (pack 5: B/32 waves, its roles alternating
// over the SIMDs), above it the packed pair; the packed split (pack 4: B/64 waves) is the
// rollout's, with the same bound.  FR3, HIP graph (profiles/r06/mix/): 32768 3.53 us (pack 5)
// / 3.99 (4); 65536 4.15 (5) / 4.24 (4); 131072 5.45 (5) / 5.50 (4).
constexpr uint32_t kSplitMaxBatch = 1u << 17;

// The forward-dynamics kernel a launch of B configurations takes (auto policy when the
// tuning `pack` is unset).
int fd_pack(const Multibody *mb, bool f64, uint32_t B) {
    int pack = 0;
    if (rbamd::tuning().pack < 0) {
        if (!f64 && rbamd::jit_fd_form(mb->model) == 2 && mb->model.n <= 8 &&
            mb->model.serial_revolute())  // splits: serial chains, measured on FR3
            pack = B <= kSplitMaxBatch ? 5 : 0;
        else  // paired lanes halve the grid: below kPackMinBatch one per lane fills more CUs
            pack = B < kPackMinBatch ? 1 : 0;
    }
    return pack;
}

const rbamd::JitKernel *jit_fd(const Multibody *mb, bool f64, uint32_t B) {
    return jit_shaped(mb, rbamd::JitKind::Fd, f64, B, false);
}

// The rollout kernel a launch of B configurations takes: fp32 mass-matrix rollouts up to 2^17
// configurations split every step over a pair of packed waves (aba_body.hip.hpp
// rollout_split_block2), as jit_fd's small-batch forward dynamics.  FR3, K = 16, HIP graph:
// 16384 43.3 vs 62.7 us (pair), 65536 43.6 vs 63.5, 131072 58.9 vs 63.7; 262144 101.5 vs 93.2
// (profiles/r03/rollout_split/).
int rollout_pack(const Multibody *mb, bool f64, uint32_t B) {
    return (rbamd::tuning().pack < 0 && !f64 && B <= kSplitMaxBatch &&
            rbamd::jit_fd_form(mb->model, rbamd::JitKind::Rollout) == 2 &&
            !(rbamd::tuning().jit_variant & 256)) ? 4 : 0;
}

const rbamd::JitKernel *jit_rollout(const Multibody *mb, bool f64, uint32_t B) {
    return jit_shaped(mb, rbamd::JitKind::Rollout, f64, B, false);
}

int idfd_pack(bool f64, uint32_t B);

JitShape jit_shape(const Multibody *mb, rbamd::JitKind kind, bool f64, uint32_t B, bool tiled) {
    JitShape sh;
    switch (kind) {
        case rbamd::JitKind::Rnea: sh = rnea_shape(mb, f64, B, tiled); break;
        case rbamd::JitKind::Fd: sh.pack = fd_pack(mb, f64, B); break;
        case rbamd::JitKind::Rollout: sh.pack = rollout_pack(mb, f64, B); break;
        case rbamd::JitKind::RneaFd: sh.pack = idfd_pack(f64, B); break;
        default: break;
    }
    // CRBA evaluates its angles with the precise fp32 sincos; every other kind with the fast one
    // unless RB_FAST_TRIG=0 (fp64 always its own)
    sh.fast = kind != rbamd::JitKind::Crba && fast_trig() && !f64;
    return sh;
}

unsigned jit_grid(const rbamd::JitKernel *jk, uint32_t B) {
    if (jk->pack == 3 && jk->seq_tail > 0) {  // pairs, then a one-per-lane tail (jit.cpp)
        const unsigned T = (unsigned)(((uint64_t)B + 255u) / 256u);
        const unsigned S = (unsigned)(((uint64_t)T * (unsigned)jk->seq_tail) / 100u);
        const unsigned P = (T - S) & ~1u;
        return P / 2u + (T - P);
    }
    // pack 2 / 3: two configurations per lane; pack 5: the one-per-lane wave split, 128 per block
    // (pack 4, the packed split, covers 256 per block like one per lane)
    const unsigned per_block = jk->pack == 5 ? 128u : 256u * ((jk->pack == 2 || jk->pack == 3) ? 2u : 1u);
    return (unsigned)(((uint64_t)B + per_block - 1) / per_block);
}

hipError_t jit_launch(const rbamd::JitKernel *jk, uint32_t B, void **args, hipStream_t s) {
    return hipModuleLaunchKernel(jk->function, jit_grid(jk, B), 1, 1, jk->block, 1, 1, 0, s, args, nullptr);
}

// tiled: the [ceil(B/256)][n][256] layout (kernels.hpp); the JIT lane kernels and the
// generic lane kernels take it through their block stride (the generic grid-stride RNEA is
// SoA-only and never chosen for it).
template <typename T>
hipError_t launch_rnea_any(const Multibody *mb, const T *mdl, const T *q, const T *qd, const T *qdd, T *tau,
                           uint32_t B, int64_t ld, hipStream_t s, bool tiled = false) {
    if (B == 0) return hipSuccess;
    if (const rbamd::JitKernel *jk = jit_rnea(mb, sizeof(T) == 8, B, tiled)) {
        const int64_t lda = tiled ? 256 : ld, bs = tiled ? (int64_t)mb->model.n * 256 : 256;
        void *args[] = {(void *)&q, (void *)&qd, (void *)&qdd, (void *)&tau, (void *)&B, (void *)&lda, (void *)&bs};
        return jit_launch(jk, B, args, s);
    }
    if (!mb->model.serial_revolute()) return no_generic(mb);
    return rbamd::launch_rnea<T>(mb->model.n, mdl, q, qd, qdd, tau, B, ld, s, fast_trig(), tiled);
}

template <typename T>
hipError_t launch_fd_any(const Multibody *mb, const T *mdl, const T *q, const T *qd, const T *tau, T *qdd,
                         uint32_t B, int64_t ld, hipStream_t s, bool tiled = false) {
    if (B == 0) return hipSuccess;
    if (const rbamd::JitKernel *jk = jit_fd(mb, sizeof(T) == 8, B)) {
        const int64_t lda = tiled ? 256 : ld, bs = tiled ? (int64_t)mb->model.n * 256 : 256;
        void *args[] = {(void *)&q, (void *)&qd, (void *)&tau, (void *)&qdd, (void *)&B, (void *)&lda, (void *)&bs};
        return jit_launch(jk, B, args, s);
    }
    if (!mb->model.serial_revolute()) return no_generic(mb);
    return rbamd::launch_aba<T>(mb->model.n, mdl, q, qd, tau, qdd, B, ld, s, fast_trig(), tiled);
}

// Inverse + forward dynamics of the same (q, qd) (config 4's pair): one fused hipRTC launch
// (fdh_body.hip.hpp idfd_lane) for models on the mass-matrix forward dynamics; otherwise -- the
// ABA models (trees, chains over 12 links), hipRTC off or failed -- the RNEA launch then the
// forward-dynamics launch, the same results.
// The fused pair's kernel form for B configurations (auto policy when the tuning `pack` is
// unset): the wave split (pack 5, idfd_split_block1) for fp32 up to 2^16 configurations, one
// per lane otherwise.  FR3, HIP graph, tiled (profiles/r06/split/): fp32 65536 4.82 vs 5.24 us,
// 131072 6.79 vs 6.49; fp64 65536 6.64 vs 6.70, 131072 11.55 vs 10.67, 262144 22.06 vs 20.59 --
// as for the forward dynamics alone (fp64 FD split 10.16 vs 8.62 us at 2^17): the SIMDs already
// hold 2 waves of the one-per-lane kernel there, and the split repeats the loads and sincos.
// With the split's roles alternating over the SIMDs (round 6, profiles/r06/mix/): fp32 65536
// 4.75 us, 131072 6.53 vs 6.46 one per lane -- the bound stays.
constexpr uint32_t kIdfdSplitMaxBatch32 = 1u << 16;
int idfd_pack(bool f64, uint32_t B) {
    if (rbamd::tuning().pack >= 0) return 0;
    return (!f64 && B <= kIdfdSplitMaxBatch32) ? 5 : 1;
}

const rbamd::JitKernel *jit_idfd(const Multibody *mb, bool f64, uint32_t B) {
    if (!mb->model.serial_revolute() || rbamd::jit_fd_form(mb->model, rbamd::JitKind::RneaFd) != 2) return nullptr;
    return jit_shaped(mb, rbamd::JitKind::RneaFd, f64, B, false);
}

template <typename T>
hipError_t launch_idfd_any(const Multibody *mb, const T *mdl, const T *q, const T *qd, const T *qdd, const T *tau_in,
                           T *tau, T *qdd_out, uint32_t B, int64_t ld, hipStream_t s, bool tiled = false) {
    if (B == 0) return hipSuccess;
    if (const rbamd::JitKernel *jk = jit_idfd(mb, sizeof(T) == 8, B)) {
        const int64_t lda = tiled ? 256 : ld, bs = tiled ? (int64_t)mb->model.n * 256 : 256;
        void *args[] = {(void *)&q,   (void *)&qd, (void *)&qdd,  (void *)&tau_in, (void *)&tau,
                        (void *)&qdd_out, (void *)&B, (void *)&lda, (void *)&bs};
        return jit_launch(jk, B, args, s);
    }
    hipError_t e = launch_rnea_any<T>(mb, mdl, q, qd, qdd, tau, B, ld, s, tiled);
    if (e != hipSuccess) return e;
    return launch_fd_any<T>(mb, mdl, q, qd, tau_in, qdd_out, B, ld, s, tiled);
}

template <typename T>
hipError_t launch_rollout_any(const Multibody *mb, const T *mdl, T *q, T *qd, const T *tau_seq, T dt, int K, T *traj,
                              uint32_t B, int64_t ld, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (const rbamd::JitKernel *jk = jit_rollout(mb, sizeof(T) == 8, B)) {
        void *args[] = {(void *)&q, (void *)&qd, (void *)&tau_seq, (void *)&dt, (void *)&K, (void *)&traj,
                        (void *)&B, (void *)&ld};
        return jit_launch(jk, B, args, s);
    }
    if (!mb->model.serial_revolute()) return no_generic(mb);
    return rbamd::launch_rollout<T>(mb->model.n, mdl, q, qd, tau_seq, dt, K, traj, B, ld, s, fast_trig());
}

template <typename T>
hipError_t launch_crba_any(const Multibody *mb, const T *mdl, const T *q, T *H, uint32_t B, int64_t ld,
                           hipStream_t s, bool tiled = false) {
    if (B == 0) return hipSuccess;
    if (const rbamd::JitKernel *jk = jit_get(mb, rbamd::JitKind::Crba, sizeof(T) == 8, false)) {
        const int64_t n = mb->model.n, lda = tiled ? 256 : ld, bs_in = tiled ? n * 256 : 256,
                      bs_out = tiled ? n * n * 256 : 256;
        void *args[] = {(void *)&q, (void *)&H, (void *)&B, (void *)&lda, (void *)&bs_in, (void *)&bs_out};
        return jit_launch(jk, B, args, s);
    }
    if (!mb->model.serial_revolute()) return no_generic(mb);
    return rbamd::launch_crba<T>(mb->model.n, mdl, q, H, B, ld, s, tiled);
}

// fwd_kin / jac: the hipRTC kernels (tree_body.hip.hpp fwd_kin_tree / jac_tree, the model's
// topology and constants compiled in) for every model; serial revolute chains fall back to the
// precompiled kernels (kinematics.hip) when hipRTC is off or failed.  FR3 2^20: fwd_kin fp64
// 18.2 vs 26.4 us precompiled, fp32 9.6 vs 11.3; the Jacobian is store-bound, equal (89.2 vs
// 89.5 / 41.4 vs 41.3 us; profiles/r04/ab/ab_fk*.log, ab_jac*.log).  The launchers and
// multibody_kernel_path_ex resolve through this one.
const rbamd::JitKernel *jit_kin(const Multibody *mb, bool jac, bool f64) {
    return jit_get(mb, jac ? rbamd::JitKind::Jac : rbamd::JitKind::FwdKin, f64, !f64 && fast_trig());
}

// Serial revolute chains take the precompiled kinematics kernels only when the (experimental)
// tuning `kin_jit` is 0.
bool kin_precompiled(const Multibody *mb) {
    return mb->model.serial_revolute() && rbamd::tuning().kin_jit == 0;
}

template <typename T>
hipError_t launch_kin_any(const Multibody *mb, bool jac, const T *mdl, const T *q, T *out, uint32_t B, int64_t ld,
                          hipStream_t s, bool tiled = false) {
    if (B == 0) return hipSuccess;
    const bool fast = sizeof(T) == 4 && fast_trig();
    const rbamd::JitKernel *jk = kin_precompiled(mb) ? nullptr : jit_kin(mb, jac, sizeof(T) == 8);
    if (!jk && mb->model.serial_revolute())
        return jac ? rbamd::launch_jac<T>(mb->model.n, mdl, q, out, B, ld, s, fast, tiled)
                   : rbamd::launch_fwd_kin<T>(mb->model.n, mdl, q, out, B, ld, s, fast, tiled);
    if (!jk) return no_generic(mb);
    const int64_t n = mb->model.n, lda = tiled ? 256 : ld, bs_in = tiled ? n * 256 : 256,
                  bs_out = tiled ? (jac ? 6 * n : 3) * 256 : 256;
    void *args[] = {(void *)&q, (void *)&out, (void *)&B, (void *)&lda, (void *)&bs_in, (void *)&bs_out};
    return jit_launch(jk, B, args, s);
}

constexpr int64_t kChunk = int64_t(1) << 28;  // per-launch batch cap: b * sizeof(T) < 2^32

int check_batch(const Multibody *mb, int64_t batch, int64_t ld) {
    if (!mb) return set_err(RB_ERR_NULL, "NULL Multibody handle");
    if (batch < 0) return set_err(RB_ERR_ARG, "negative batch");
    if (ld < batch) return set_err(RB_ERR_ARG, "leading dimension ld < batch");
    return RB_OK;
}

// Thread-local staging for the single-configuration ABI: one stream, one device
// buffer and one pinned host buffer per thread and device (never freed: HIP teardown
// order at process exit is not ours to control).
struct Staging {
    hipStream_t stream = nullptr;
    double *dbuf = nullptr;
    size_t dcap = 0;
    double *hbuf = nullptr;
    size_t hcap = 0;
};
thread_local std::map<int, Staging> t_staging;

int staging(size_t doubles, Staging **out) {
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return hip_err(e, "hipGetDevice");
    Staging &s = t_staging[d];
    if (!s.stream) {
        if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
            return hip_err(e, "hipStreamCreate");
    }
    if (s.dcap < doubles) {
        if (s.dbuf) (void)hipFree(s.dbuf);
        s.dbuf = nullptr;
        s.dcap = 0;
        if ((e = hipMalloc(&s.dbuf, doubles * sizeof(double))) != hipSuccess) return hip_err(e, "hipMalloc");
        s.dcap = doubles;
    }
    if (s.hcap < doubles) {
        if (s.hbuf) (void)hipHostFree(s.hbuf);
        s.hbuf = nullptr;
        s.hcap = 0;
        if ((e = hipHostMalloc(&s.hbuf, doubles * sizeof(double), hipHostMallocDefault)) != hipSuccess)
            return hip_err(e, "hipHostMalloc");
        s.hcap = doubles;
    }
    *out = &s;
    return RB_OK;
}

// Host evaluation of one single-configuration query (host_eval.cpp) when the model and CPU
// allow it and the caller has not asked for the GPU (tuning single_gpu); `eval(out)` fills
// the result.  Returns the malloc'd result, or nullptr with *used = false to take the GPU.
template <typename F>
double *single_host(const Multibody *mb, const double *const *inputs, int nin, size_t nout, bool *used, F eval) {
    *used = false;
    if (!mb || rbamd::tuning().single_gpu != 0 || !rbamd::host_eval_supported(mb->model)) return nullptr;
    for (int k = 0; k < nin; ++k)
        if (!inputs[k]) { set_err(RB_ERR_NULL, "NULL input vector"); *used = true; return nullptr; }
    *used = true;
    double *res = static_cast<double *>(std::malloc(nout * sizeof(double)));
    if (!res) { set_err(RB_ERR_ARG, "out of host memory"); return nullptr; }
    if (!eval(res)) { std::free(res); *used = false; return nullptr; }
    return res;
}

// Runs one single-configuration query on the GPU: `nin` input vectors of n doubles,
// `nout` output doubles; `launch(dev_in, dev_out, stream)` enqueues the kernel.
template <typename F>
double *single_query(const Multibody *mb, const double *const *inputs, int nin, size_t nout, F launch) {
    if (!mb) { set_err(RB_ERR_NULL, "NULL Multibody handle"); return nullptr; }
    const int n = mb->model.n;
    for (int k = 0; k < nin; ++k)
        if (!inputs[k]) { set_err(RB_ERR_NULL, "NULL input vector"); return nullptr; }
    Staging *s = nullptr;
    const size_t total = (size_t)nin * n + nout;
    if (staging(total, &s) != RB_OK) return nullptr;
    for (int k = 0; k < nin; ++k) std::memcpy(s->hbuf + (size_t)k * n, inputs[k], n * sizeof(double));
    hipError_t e = hipMemcpyAsync(s->dbuf, s->hbuf, (size_t)nin * n * sizeof(double), hipMemcpyHostToDevice, s->stream);
    if (e != hipSuccess) { hip_err(e, "hipMemcpyAsync H2D"); return nullptr; }
    int rc = launch(s->dbuf, s->dbuf + (size_t)nin * n, s->stream);
    if (rc != RB_OK) return nullptr;
    e = hipMemcpyAsync(s->hbuf + (size_t)nin * n, s->dbuf + (size_t)nin * n, nout * sizeof(double), hipMemcpyDeviceToHost, s->stream);
    if (e != hipSuccess) { hip_err(e, "hipMemcpyAsync D2H"); return nullptr; }
    if ((e = hipStreamSynchronize(s->stream)) != hipSuccess) { hip_err(e, "hipStreamSynchronize"); return nullptr; }
    double *res = static_cast<double *>(std::malloc(nout * sizeof(double)));
    if (!res) { set_err(RB_ERR_ARG, "out of host memory"); return nullptr; }
    std::memcpy(res, s->hbuf + (size_t)nin * n, nout * sizeof(double));
    return res;
}

template <typename T, typename L>
int chunked(int64_t batch, L &&one) {
    for (int64_t b0 = 0; b0 < batch; b0 += kChunk) {
        const int64_t nb = batch - b0 < kChunk ? batch - b0 : kChunk;
        int rc = one(b0, (uint32_t)nb);
        if (rc != RB_OK) return rc;
    }
    return RB_OK;
}

template <typename T>
int rnea_batch(const Multibody *mb, const T *q, const T *qd, const T *qdd, T *tau, int64_t batch,
               int64_t ld, void *stream, bool tiled = false) {
    int rc = check_batch(mb, batch, tiled ? batch : ld);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    if (!q || !qd || !qdd || !tau) return set_err(RB_ERR_NULL, "NULL array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    const int64_t per = tiled ? mb->model.n : 1;  // element offset of configuration b0 (b0 % 256 == 0)
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        const int64_t o = b0 * per;
        hipError_t e = launch_rnea_any<T>(mb, mdl, q + o, qd + o, qdd + o, tau + o, nb, ld, (hipStream_t)stream, tiled);
        return e == hipSuccess ? RB_OK : hip_err(e, "rnea launch");
    });
}

template <typename T>
int fd_batch(const Multibody *mb, const T *q, const T *qd, const T *tau, T *qdd, int64_t batch,
             int64_t ld, void *stream, bool tiled = false) {
    int rc = check_batch(mb, batch, tiled ? batch : ld);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    if (!q || !qd || !tau || !qdd) return set_err(RB_ERR_NULL, "NULL array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    const int64_t per = tiled ? mb->model.n : 1;
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        const int64_t o = b0 * per;
        hipError_t e = launch_fd_any<T>(mb, mdl, q + o, qd + o, tau + o, qdd + o, nb, ld, (hipStream_t)stream, tiled);
        return e == hipSuccess ? RB_OK : hip_err(e, "aba launch");
    });
}

template <typename T>
int idfd_batch(const Multibody *mb, const T *q, const T *qd, const T *qdd, const T *tau_in, T *tau, T *qdd_out,
               int64_t batch, int64_t ld, void *stream, bool tiled = false) {
    int rc = check_batch(mb, batch, tiled ? batch : ld);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    if (!q || !qd || !qdd || !tau_in || !tau || !qdd_out) return set_err(RB_ERR_NULL, "NULL array");
    // outputs must not overlap the inputs (the kernel reads tau_in after storing tau); the exact
    // aliases a caller is likely to pass -- tau_in as tau, qdd as qdd_out -- are refused here
    for (const T *o : {(const T *)tau, (const T *)qdd_out})
        for (const T *i : {q, qd, qdd, tau_in})
            if (o == i) return set_err(RB_ERR_ARG, "rnea_fd: an output array is also an input (no in-place form)");
    if (tau == qdd_out) return set_err(RB_ERR_ARG, "rnea_fd: tau and qdd_out are the same array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    const int64_t per = tiled ? mb->model.n : 1;
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        const int64_t o = b0 * per;
        hipError_t e = launch_idfd_any<T>(mb, mdl, q + o, qd + o, qdd + o, tau_in + o, tau + o, qdd_out + o, nb, ld,
                                          (hipStream_t)stream, tiled);
        return e == hipSuccess ? RB_OK : hip_err(e, "rnea_fd launch");
    });
}

template <typename T>
int rollout_batch(const Multibody *mb, T *q, T *qd, const T *tau_seq, double dt, int K, T *traj, int64_t batch,
                  int64_t ld, void *stream) {
    int rc = check_batch(mb, batch, ld);
    if (rc) return rc;
    if (K < 0) return set_err(RB_ERR_ARG, "negative step count");
    if (batch == 0 || K == 0) return RB_OK;
    if (!q || !qd || !tau_seq) return set_err(RB_ERR_NULL, "NULL array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        hipError_t e = launch_rollout_any<T>(mb, mdl, q + b0, qd + b0, tau_seq + b0, (T)dt, K,
                                             traj ? traj + b0 : nullptr, nb, ld, (hipStream_t)stream);
        return e == hipSuccess ? RB_OK : hip_err(e, "rollout launch");
    });
}

template <typename T>
int crba_batch(const Multibody *mb, const T *q, T *H, int64_t batch, int64_t ld, void *stream, bool tiled = false) {
    int rc = check_batch(mb, batch, tiled ? batch : ld);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    if (!q || !H) return set_err(RB_ERR_NULL, "NULL array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    // element offsets of configuration b0 (b0 % 256 == 0) in the input / output arrays
    const int64_t n = mb->model.n, pin = tiled ? n : 1, pout = tiled ? n * n : 1;
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        hipError_t e = launch_crba_any<T>(mb, mdl, q + b0 * pin, H + b0 * pout, nb, ld, (hipStream_t)stream, tiled);
        return e == hipSuccess ? RB_OK : hip_err(e, "crba launch");
    });
}

template <typename T>
int kin_batch(const Multibody *mb, bool jac, const T *q, T *out, int64_t batch, int64_t ld, void *stream,
              bool tiled = false) {
    int rc = check_batch(mb, batch, tiled ? batch : ld);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    if (!q || !out) return set_err(RB_ERR_NULL, "NULL array");
    const T *mdl = nullptr;
    if ((rc = device_consts<T>(mb, &mdl))) return rc;
    const int64_t n = mb->model.n, pin = tiled ? n : 1, pout = tiled ? (jac ? 6 * n : 3) : 1;
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        hipError_t e = launch_kin_any<T>(mb, jac, mdl, q + b0 * pin, out + b0 * pout, nb, ld, (hipStream_t)stream, tiled);
        return e == hipSuccess ? RB_OK : hip_err(e, jac ? "jac launch" : "fwd_kin launch");
    });
}

Multibody *new_from_text(const std::string &xml, unsigned flags = 0) {
    try {
        return make(rbamd::Model::from_urdf_text(xml, flags));
    } catch (const std::exception &ex) {
        set_err(RB_ERR_URDF, ex.what());
        return nullptr;
    }
}

}  // namespace

namespace {
// nin input and nout output [n][batch] host arrays; launch(d_in, d_out, stream) gets the device
// copies of the inputs (consecutive) and room for the outputs (consecutive).
template <typename T, typename Launch>
int host_batch(const Multibody *mb, const T *const *in, int nin, T *const *out, int nout, int64_t batch,
               Launch launch) {
    int rc = check_batch(mb, batch, batch);
    if (rc) return rc;
    if (batch == 0) return RB_OK;
    for (int k = 0; k < nin; ++k)
        if (!in[k]) return set_err(RB_ERR_NULL, "NULL array");
    for (int k = 0; k < nout; ++k)
        if (!out[k]) return set_err(RB_ERR_NULL, "NULL array");
    const size_t per = (size_t)mb->model.n * (size_t)batch;
    T *d = nullptr;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_err(e, "hipStreamCreate");
    e = hipMallocAsync((void **)&d, per * (nin + nout) * sizeof(T), s);
    if (e != hipSuccess) { (void)hipStreamDestroy(s); return hip_err(e, "hipMallocAsync"); }
    for (int k = 0; k < nin && e == hipSuccess; ++k)
        e = hipMemcpyAsync(d + k * per, in[k], per * sizeof(T), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) rc = launch(d, d + nin * per, s);
    else rc = hip_err(e, "hipMemcpyAsync H2D");
    for (int k = 0; k < nout && rc == RB_OK; ++k) {
        e = hipMemcpyAsync(out[k], d + (nin + k) * per, per * sizeof(T), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) rc = hip_err(e, "hipMemcpyAsync D2H");
    }
    (void)hipFreeAsync(d, s);
    e = hipStreamSynchronize(s);
    if (rc == RB_OK && e != hipSuccess) rc = hip_err(e, "hipStreamSynchronize");
    (void)hipStreamDestroy(s);
    return rc;
}
// Blocking host-pointer forms: SoA rows x[j * batch + b] in host memory, copied to a scratch
// device buffer on a private stream, evaluated by the batched kernels, copied back.
template <typename T>
int rnea_host(const Multibody *mb, const T *q, const T *qd, const T *qdd, T *tau, int64_t batch) {
    const T *in[3] = {q, qd, qdd};
    T *out[1] = {tau};
    return host_batch<T>(mb, in, 3, out, 1, batch, [&](T *d, T *o, hipStream_t s) {
        const size_t per = (size_t)mb->model.n * (size_t)batch;
        return rnea_batch<T>(mb, d, d + per, d + 2 * per, o, batch, batch, s);
    });
}
template <typename T>
int fd_host(const Multibody *mb, const T *q, const T *qd, const T *tau, T *qdd, int64_t batch) {
    const T *in[3] = {q, qd, tau};
    T *out[1] = {qdd};
    return host_batch<T>(mb, in, 3, out, 1, batch, [&](T *d, T *o, hipStream_t s) {
        const size_t per = (size_t)mb->model.n * (size_t)batch;
        return fd_batch<T>(mb, d, d + per, d + 2 * per, o, batch, batch, s);
    });
}
template <typename T>
int idfd_host(const Multibody *mb, const T *q, const T *qd, const T *qdd, const T *tau_in, T *tau, T *qdd_out,
              int64_t batch) {
    const T *in[4] = {q, qd, qdd, tau_in};
    T *out[2] = {tau, qdd_out};
    return host_batch<T>(mb, in, 4, out, 2, batch, [&](T *d, T *o, hipStream_t s) {
        const size_t per = (size_t)mb->model.n * (size_t)batch;
        return idfd_batch<T>(mb, d, d + per, d + 2 * per, d + 3 * per, o, o + per, batch, batch, s);
    });
}
}  // namespace

namespace {
template <typename T>
int fill_uniform(T *x, int rows, int64_t batch, int64_t ld, const double *lo, const double *hi, uint64_t seed,
                 void *stream) {
    if (!x || !lo || !hi) return set_err(RB_ERR_NULL, "NULL argument");
    if (rows < 1 || batch < 0 || ld < batch) return set_err(RB_ERR_ARG, "bad fill shape");
    // one launch; the generator's lane index is 32-bit (b * sizeof(T) < 2^32 as the dynamics)
    if (batch > kChunk) return set_err(RB_ERR_ARG, "fill batch above 2^28 configurations not supported");
    if (batch == 0) return RB_OK;
    hipStream_t s = (hipStream_t)stream;
    std::vector<double> lohi(2 * (size_t)rows);
    for (int j = 0; j < rows; ++j) {
        lohi[2 * j] = lo[j];
        lohi[2 * j + 1] = hi[j];
    }
    double *d = nullptr;
    hipError_t e = hipMallocAsync((void **)&d, lohi.size() * sizeof(double), s);
    if (e != hipSuccess) return hip_err(e, "hipMallocAsync");
    e = hipMemcpyAsync(d, lohi.data(), lohi.size() * sizeof(double), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return hip_err(e, "hipMemcpyAsync");
    int rc = RB_OK;
    e = rbamd::launch_fill_uniform<T>(x, rows, (uint32_t)batch, ld, d, seed, s);
    if (e != hipSuccess) rc = hip_err(e, "fill launch");
    (void)hipFreeAsync(d, s);
    // the host-side lohi vector dies here; make sure the copy has consumed it
    e = hipStreamSynchronize(s);
    if (rc == RB_OK && e != hipSuccess) rc = hip_err(e, "hipStreamSynchronize");
    return rc;
}
}  // namespace

extern "C" {

// ------------------------------------------------------------- reference ABI (6)
Multibody *multibody_new(void) {
    if (const char *path = std::getenv("RIGIDBODY_URDF")) {
        if (*path) return multibody_new_from_urdf(path);
    }
    return new_from_text(std::string(kFr3Urdf));
}

void multibody_free(Multibody *mb) {
    if (!mb) return;
    int cur = 0;
    bool have_cur = hipGetDevice(&cur) == hipSuccess;
    for (auto &kv : mb->dev) {
        if (hipSetDevice(kv.first) != hipSuccess) continue;
        if (kv.second.f32) (void)hipFree(kv.second.f32);
        if (kv.second.f64) (void)hipFree(kv.second.f64);
    }
    for (auto &kv : mb->jit) {
        if (!kv.second.module) continue;
        if (hipSetDevice(mb->jit_device[kv.first]) != hipSuccess) continue;
        (void)hipModuleUnload(kv.second.module);
    }
    if (have_cur) (void)hipSetDevice(cur);
    delete mb;
}

double *multibody_rnea(const Multibody *mb, const double *q, const double *dq, const double *ddq) {
    const double *in[3] = {q, dq, ddq};
    const size_t n = mb ? (size_t)mb->model.n : 0;
    bool host = false;
    double *r = single_host(mb, in, 3, n, &host, [&](double *o) {
        return rbamd::host_rnea(mb->model, mb->pk64.data(), q, dq, ddq, o);
    });
    if (host) return r;
    return single_query(mb, in, 3, n, [&](double *din, double *dout, hipStream_t s) {
        const double *mdl = nullptr;
        int rc = device_consts<double>(mb, &mdl);
        if (rc) return rc;
        hipError_t e = launch_rnea_any<double>(mb, mdl, din, din + n, din + 2 * n, dout, 1, 1, s);
        return e == hipSuccess ? RB_OK : hip_err(e, "rnea launch");
    });
}

double *multibody_crba(const Multibody *mb, const double *q) {
    const double *in[1] = {q};
    const size_t n = mb ? (size_t)mb->model.n : 0;
    bool host = false;
    double *r = single_host(mb, in, 1, n * n, &host, [&](double *o) {
        return rbamd::host_crba(mb->model, mb->pk64.data(), q, o);
    });
    if (host) return r;
    return single_query(mb, in, 1, n * n, [&](double *din, double *dout, hipStream_t s) {
        const double *mdl = nullptr;
        int rc = device_consts<double>(mb, &mdl);
        if (rc) return rc;
        hipError_t e = launch_crba_any<double>(mb, mdl, din, dout, 1, 1, s);
        return e == hipSuccess ? RB_OK : hip_err(e, "crba launch");
    });
}

double *multibody_fwd_kin(const Multibody *mb, const double *q) {
    const double *in[1] = {q};
    bool host = false;
    double *r = single_host(mb, in, 1, 3, &host, [&](double *o) {
        return rbamd::host_fwd_kin(mb->model, mb->pk64.data(), q, o);
    });
    if (host) return r;
    return single_query(mb, in, 1, 3, [&](double *din, double *dout, hipStream_t s) {
        const double *mdl = nullptr;
        int rc = device_consts<double>(mb, &mdl);
        if (rc) return rc;
        hipError_t e = launch_kin_any<double>(mb, false, mdl, din, dout, 1, 1, s);
        return e == hipSuccess ? RB_OK : hip_err(e, "fwd_kin launch");
    });
}

double *multibody_jac(const Multibody *mb, const double *q) {
    const double *in[1] = {q};
    const size_t n = mb ? (size_t)mb->model.n : 0;
    bool host = false;
    double *r = single_host(mb, in, 1, 6 * n, &host, [&](double *o) {
        return rbamd::host_jac(mb->model, mb->pk64.data(), q, o);
    });
    if (host) return r;
    return single_query(mb, in, 1, 6 * n, [&](double *din, double *dout, hipStream_t s) {
        const double *mdl = nullptr;
        int rc = device_consts<double>(mb, &mdl);
        if (rc) return rc;
        hipError_t e = launch_kin_any<double>(mb, true, mdl, din, dout, 1, 1, s);
        return e == hipSuccess ? RB_OK : hip_err(e, "jac launch");
    });
}

// ---------------------------------------------------------------- model handling
Multibody *multibody_new_from_urdf_ex(const char *path, unsigned flags) {
    if (!path) { set_err(RB_ERR_NULL, "NULL path"); return nullptr; }
    std::ifstream f(path, std::ios::binary);
    if (!f) { set_err(RB_ERR_URDF, std::string("cannot open URDF: ") + path); return nullptr; }
    std::stringstream ss;
    ss << f.rdbuf();
    return new_from_text(ss.str(), flags);
}

Multibody *multibody_new_from_urdf_string_ex(const char *xml, size_t len, unsigned flags) {
    if (!xml) { set_err(RB_ERR_NULL, "NULL URDF string"); return nullptr; }
    return new_from_text(std::string(xml, len), flags);
}

Multibody *multibody_new_from_urdf(const char *path) { return multibody_new_from_urdf_ex(path, 0); }

Multibody *multibody_new_from_urdf_string(const char *xml, size_t len) {
    return multibody_new_from_urdf_string_ex(xml, len, 0);
}

unsigned multibody_flags(const Multibody *mb) {
    if (!mb) { set_err(RB_ERR_NULL, "NULL Multibody handle"); return 0u; }
    return mb->model.flags;
}

int64_t multibody_blob_size(const Multibody *mb) {
    if (!mb) return -set_err(RB_ERR_NULL, "NULL Multibody handle");
    return rbamd::kBlobHeader + (int64_t)mb->model.n * rbamd::kBlobPerLink;
}

int multibody_export_blob(const Multibody *mb, double *out, int64_t len) {
    if (!mb || !out) return set_err(RB_ERR_NULL, "NULL argument");
    std::vector<double> b = mb->model.blob();
    if (len < (int64_t)b.size()) return set_err(RB_ERR_ARG, "blob buffer too small");
    std::memcpy(out, b.data(), b.size() * sizeof(double));
    return RB_OK;
}

Multibody *multibody_new_from_blob(const double *blob, int64_t len) {
    try {
        return make(rbamd::Model::from_blob(blob, len));
    } catch (const std::exception &ex) {
        set_err(RB_ERR_ARG, ex.what());
        return nullptr;
    }
}

int multibody_dof(const Multibody *mb) { return mb ? mb->model.n : -set_err(RB_ERR_NULL, "NULL Multibody handle"); }

double multibody_total_mass(const Multibody *mb) {
    if (!mb) { set_err(RB_ERR_NULL, "NULL Multibody handle"); return std::nan(""); }
    return mb->model.total_mass();
}

int multibody_limits(const Multibody *mb, double *lower, double *upper, double *velocity, double *effort) {
    if (!mb) return set_err(RB_ERR_NULL, "NULL Multibody handle");
    for (int i = 0; i < mb->model.n; ++i) {
        const rbamd::LinkModel &L = mb->model.links[i];
        if (lower) lower[i] = L.lower;
        if (upper) upper[i] = L.upper;
        if (velocity) velocity[i] = L.velocity;
        if (effort) effort[i] = L.effort;
    }
    return RB_OK;
}

int multibody_supported_dofs(int *out, int cap) { return rbamd::supported_dofs(out, cap); }

int multibody_topology(const Multibody *mb, int *parent, int *joint_type) {
    if (!mb) return set_err(RB_ERR_NULL, "NULL Multibody handle");
    for (int i = 0; i < mb->model.n; ++i) {
        if (parent) parent[i] = mb->model.links[i].parent;
        if (joint_type) joint_type[i] = mb->model.links[i].type;
    }
    return RB_OK;
}

}  // extern "C"

// C++ helpers of the kernel-inspection entry points below
namespace {
// The kernel a launch of `batch` configurations of `kind` takes: the same resolution as the
// launchers (launch_*_any).  *generic = true when the precompiled kernel runs (serial revolute
// fwd_kin / jac, JIT disabled or failed).
const rbamd::JitKernel *resolve_kernel(const Multibody *mb, int kind, bool f64, int64_t batch, bool tiled) {
    if ((kind == 4 || kind == 5) && kin_precompiled(mb)) return nullptr;  // precompiled kinematics
    if (!rbamd::jit_enabled()) return nullptr;
    const uint32_t B = batch < kChunk ? (uint32_t)batch : (uint32_t)kChunk;
    if (kind == 0) return jit_rnea(mb, f64, B, tiled);
    if (kind == 1) return jit_fd(mb, f64, B);
    if (kind == 3) return jit_rollout(mb, f64, B);
    if (kind == 6) return jit_idfd(mb, f64, B);
    if (kind >= 4) return jit_kin(mb, kind == 5, f64);
    return jit_get(mb, rbamd::JitKind::Crba, f64, false);
}

int check_kernel_query(const Multibody *mb, int kind, int64_t batch) {
    if (!mb) return set_err(RB_ERR_NULL, "NULL Multibody handle");
    if (kind < 0 || kind >= rbamd::kJitKinds) return set_err(RB_ERR_ARG, kKindMsg);
    if (batch < 1) return set_err(RB_ERR_ARG, "batch must be positive");
    return RB_OK;
}

// The (pack, tail) jit_get resolves a shape to (the kernel's actual form).
void resolve_pack(const Multibody *mb, rbamd::JitKind kind, bool f64, const JitShape &sh, int *pk, int *tl) {
    *pk = sh.pack > 0 ? sh.pack : rbamd::jit_model_pack(mb->model, kind, f64, 0);
    *tl = (kind == rbamd::JitKind::Rnea && *pk == 3) ? sh.tail : 0;
}

// The hipRTC source of the kernel a launch of `batch` configurations (tiled or SoA) would run:
// compiled here (hipRTC, gfx950, no device needed) so that the occupancy-cliff rebuild of
// jit_compile shows in it -- the source of the code object a launch really loads; the generated
// source as it stands if hipRTC fails.
std::string shaped_source(const Multibody *mb, int kind, bool f64, int64_t batch, bool tiled) {
    const uint32_t B = batch < kChunk ? (uint32_t)batch : (uint32_t)kChunk;
    const auto k = (rbamd::JitKind)kind;
    const JitShape sh = jit_shape(mb, k, f64, B, tiled);
    int pk = 0, tl = 0;
    resolve_pack(mb, k, f64, sh, &pk, &tl);
    // the length query and the copy of multibody_jit_source_ex come in pairs: one compile for both
    thread_local std::string t_key, t_src;
    const std::string plain = rbamd::jit_source(mb->model, k, f64, sh.fast, pk, tl, sh.nt);
    const std::string key = std::to_string((uintptr_t)mb) + ":" + std::to_string(rbamd::tuning_generation()) + ":" + plain;
    if (key == t_key) return t_src;
    std::vector<char> code;
    std::string err, src;
    if (!rbamd::jit_compile(mb->model, k, f64, sh.fast, "gfx950", &code, &err, pk, tl, sh.nt, &src)) src = plain;
    t_key = key;
    t_src = src;
    return src;
}

void note_jit_errors(const Multibody *mb) {
    std::lock_guard<std::mutex> lk(mb->mu);
    for (auto &kv : mb->jit)
        if (!kv.second.error.empty()) g_last_error = kv.second.error;
}
}  // namespace

extern "C" {

int multibody_kernel_path_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled) {
    if (int rc = check_kernel_query(mb, kind, batch)) return -rc;
    if (resolve_kernel(mb, kind, f64 != 0, batch, tiled != 0)) return 1;
    if (rbamd::jit_enabled() && !((kind == 4 || kind == 5) && kin_precompiled(mb))) note_jit_errors(mb);
    return 0;
}

int multibody_kernel_form_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled) {
    if (int rc = check_kernel_query(mb, kind, batch)) return -rc;
    const rbamd::JitKernel *jk = resolve_kernel(mb, kind, f64 != 0, batch, tiled != 0);
    return jk ? jk->pack : 0;
}

int multibody_kernel_path(const Multibody *mb, int kind, int f64) {
    return multibody_kernel_path_ex(mb, kind, f64, int64_t(1) << 20, 0);
}

int multibody_rnea_kernel_path(const Multibody *mb, int f64) { return multibody_kernel_path(mb, 0, f64); }

int multibody_single_config_path(const Multibody *mb) {
    if (!mb) return -set_err(RB_ERR_NULL, "NULL Multibody handle");
    return (rbamd::tuning().single_gpu == 0 && rbamd::host_eval_supported(mb->model)) ? 0 : 1;
}

int multibody_jit_source(const Multibody *mb, int kind, int f64, char *buf, int64_t cap) {
    return multibody_jit_source_ex(mb, kind, f64, int64_t(1) << 20, 0, buf, cap);
}

int multibody_jit_source_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled, char *buf, int64_t cap) {
    if (int rc = check_kernel_query(mb, kind, batch)) return -rc;
    const std::string src = shaped_source(mb, kind, f64 != 0, batch, tiled != 0);
    if (buf && cap > 0) {
        const size_t n = src.size() < (size_t)(cap - 1) ? src.size() : (size_t)(cap - 1);
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return (int)src.size();
}

int64_t multibody_jit_compile(const Multibody *mb, int kind, int f64, const char *arch) {
    return multibody_jit_compile_ex(mb, kind, f64, int64_t(1) << 20, 0, arch);
}

int64_t multibody_jit_compile_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled, const char *arch) {
    if (int rc = check_kernel_query(mb, kind, batch)) return -rc;
    const uint32_t B = batch < kChunk ? (uint32_t)batch : (uint32_t)kChunk;
    const auto k = (rbamd::JitKind)kind;
    const JitShape sh = jit_shape(mb, k, f64 != 0, B, tiled != 0);
    int pk = 0, tl = 0;
    resolve_pack(mb, k, f64 != 0, sh, &pk, &tl);
    std::vector<char> code;
    std::string err;
    if (!rbamd::jit_compile(mb->model, k, f64 != 0, sh.fast, arch ? arch : "gfx950", &code, &err, pk, tl, sh.nt))
        return -set_err(RB_ERR_HIP, err);
    return (int64_t)code.size();
}

int multibody_upload(const Multibody *mb) {
    if (!mb) return set_err(RB_ERR_NULL, "NULL Multibody handle");
    const float *a = nullptr;
    const double *b = nullptr;
    int rc = device_consts<float>(mb, &a);
    if (rc) return rc;
    return device_consts<double>(mb, &b);
}

void multibody_result_free(double *p) { std::free(p); }
const char *rb_last_error(void) { return g_last_error.c_str(); }
const char *rb_version(void) { return RB_VERSION; }

}  // extern "C"

namespace {

template <typename T>
int convert_tiled(const T *src, T *dst, int64_t ld, int rows, int64_t batch, void *stream, bool to) {
    if (!src || !dst) return set_err(RB_ERR_NULL, "NULL array");
    if (rows < 0 || batch < 0 || ld < batch) return set_err(RB_ERR_ARG, "bad layout conversion shape");
    return chunked<T>(batch, [&](int64_t b0, uint32_t nb) {
        hipError_t e = to ? rbamd::launch_to_tiled<T>(src + b0, ld, dst + b0 * rows, rows, nb, (hipStream_t)stream)
                          : rbamd::launch_from_tiled<T>(src + b0 * rows, dst + b0, ld, rows, nb, (hipStream_t)stream);
        return e == hipSuccess ? RB_OK : hip_err(e, "layout conversion");
    });
}

}  // namespace

extern "C" {

int rb_to_tiled_f32(const float *src, int64_t ld, float *dst, int rows, int64_t batch, void *stream) {
    return convert_tiled<float>(src, dst, ld, rows, batch, stream, true);
}
int rb_to_tiled_f64(const double *src, int64_t ld, double *dst, int rows, int64_t batch, void *stream) {
    return convert_tiled<double>(src, dst, ld, rows, batch, stream, true);
}
int rb_from_tiled_f32(const float *src, float *dst, int64_t ld, int rows, int64_t batch, void *stream) {
    return convert_tiled<float>(src, dst, ld, rows, batch, stream, false);
}
int rb_from_tiled_f64(const double *src, double *dst, int64_t ld, int rows, int64_t batch, void *stream) {
    return convert_tiled<double>(src, dst, ld, rows, batch, stream, false);
}

int rb_set_tuning(const char *key, int value) {
    if (!key) return set_err(RB_ERR_NULL, "NULL key");
    switch (rbamd::tuning_set(key, value)) {
        case 0: return RB_OK;
        case 2: return set_err(RB_ERR_ARG, std::string("experimental tuning key (set RB_EXPERIMENTAL=1): ") + key);
        default: return set_err(RB_ERR_ARG, std::string("unknown tuning key: ") + key);
    }
}

// ------------------------------------------------------------- batched (device)
int multibody_rnea_batch_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                             float *tau, int64_t batch, int64_t ld, void *stream) {
    return rnea_batch<float>(mb, q, qd, qdd, tau, batch, ld, stream);
}
int multibody_rnea_batch_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                             double *tau, int64_t batch, int64_t ld, void *stream) {
    return rnea_batch<double>(mb, q, qd, qdd, tau, batch, ld, stream);
}
int multibody_fd_batch_f32(const Multibody *mb, const float *q, const float *qd, const float *tau,
                           float *qdd, int64_t batch, int64_t ld, void *stream) {
    return fd_batch<float>(mb, q, qd, tau, qdd, batch, ld, stream);
}
int multibody_fd_batch_f64(const Multibody *mb, const double *q, const double *qd, const double *tau,
                           double *qdd, int64_t batch, int64_t ld, void *stream) {
    return fd_batch<double>(mb, q, qd, tau, qdd, batch, ld, stream);
}
int multibody_rnea_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                   float *tau, int64_t batch, void *stream) {
    return rnea_batch<float>(mb, q, qd, qdd, tau, batch, 256, stream, true);
}
int multibody_rnea_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                   double *tau, int64_t batch, void *stream) {
    return rnea_batch<double>(mb, q, qd, qdd, tau, batch, 256, stream, true);
}
int multibody_fd_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *tau,
                                 float *qdd, int64_t batch, void *stream) {
    return fd_batch<float>(mb, q, qd, tau, qdd, batch, 256, stream, true);
}
int multibody_fd_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *tau,
                                 double *qdd, int64_t batch, void *stream) {
    return fd_batch<double>(mb, q, qd, tau, qdd, batch, 256, stream, true);
}
int multibody_rnea_fd_batch_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                const float *tau_in, float *tau, float *qdd_out, int64_t batch, int64_t ld,
                                void *stream) {
    return idfd_batch<float>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch, ld, stream);
}
int multibody_rnea_fd_batch_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                const double *tau_in, double *tau, double *qdd_out, int64_t batch, int64_t ld,
                                void *stream) {
    return idfd_batch<double>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch, ld, stream);
}
int multibody_rnea_fd_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                      const float *tau_in, float *tau, float *qdd_out, int64_t batch, void *stream) {
    return idfd_batch<float>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch, 256, stream, true);
}
int multibody_rnea_fd_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                      const double *tau_in, double *tau, double *qdd_out, int64_t batch,
                                      void *stream) {
    return idfd_batch<double>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch, 256, stream, true);
}
int multibody_rollout_batch_f32(const Multibody *mb, float *q, float *qd, const float *tau_seq, double dt, int K,
                                 float *traj, int64_t batch, int64_t ld, void *stream) {
    return rollout_batch<float>(mb, q, qd, tau_seq, dt, K, traj, batch, ld, stream);
}
int multibody_rollout_batch_f64(const Multibody *mb, double *q, double *qd, const double *tau_seq, double dt, int K,
                                 double *traj, int64_t batch, int64_t ld, void *stream) {
    return rollout_batch<double>(mb, q, qd, tau_seq, dt, K, traj, batch, ld, stream);
}
int multibody_crba_batch_f32(const Multibody *mb, const float *q, float *H, int64_t batch, int64_t ld,
                             void *stream) {
    return crba_batch<float>(mb, q, H, batch, ld, stream);
}
int multibody_crba_batch_f64(const Multibody *mb, const double *q, double *H, int64_t batch, int64_t ld,
                             void *stream) {
    return crba_batch<double>(mb, q, H, batch, ld, stream);
}

int multibody_crba_batch_tiled_f32(const Multibody *mb, const float *q, float *H, int64_t batch, void *stream) {
    return crba_batch<float>(mb, q, H, batch, 256, stream, true);
}
int multibody_crba_batch_tiled_f64(const Multibody *mb, const double *q, double *H, int64_t batch, void *stream) {
    return crba_batch<double>(mb, q, H, batch, 256, stream, true);
}
int multibody_fwd_kin_batch_tiled_f32(const Multibody *mb, const float *q, float *pos, int64_t batch, void *stream) {
    return kin_batch<float>(mb, false, q, pos, batch, 256, stream, true);
}
int multibody_fwd_kin_batch_tiled_f64(const Multibody *mb, const double *q, double *pos, int64_t batch,
                                      void *stream) {
    return kin_batch<double>(mb, false, q, pos, batch, 256, stream, true);
}
int multibody_jac_batch_tiled_f32(const Multibody *mb, const float *q, float *J, int64_t batch, void *stream) {
    return kin_batch<float>(mb, true, q, J, batch, 256, stream, true);
}
int multibody_jac_batch_tiled_f64(const Multibody *mb, const double *q, double *J, int64_t batch, void *stream) {
    return kin_batch<double>(mb, true, q, J, batch, 256, stream, true);
}

int multibody_fwd_kin_batch_f64(const Multibody *mb, const double *q, double *pos, int64_t batch,
                                int64_t ld, void *stream) {
    return kin_batch<double>(mb, false, q, pos, batch, ld, stream);
}
int multibody_jac_batch_f64(const Multibody *mb, const double *q, double *J, int64_t batch, int64_t ld,
                            void *stream) {
    return kin_batch<double>(mb, true, q, J, batch, ld, stream);
}
int multibody_fwd_kin_batch_f32(const Multibody *mb, const float *q, float *pos, int64_t batch, int64_t ld,
                                void *stream) {
    return kin_batch<float>(mb, false, q, pos, batch, ld, stream);
}
int multibody_jac_batch_f32(const Multibody *mb, const float *q, float *J, int64_t batch, int64_t ld,
                            void *stream) {
    return kin_batch<float>(mb, true, q, J, batch, ld, stream);
}

// ------------------------------------------------------------- batched (host)

int multibody_rnea_batch_host_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                  double *tau, int64_t batch) {
    return rnea_host<double>(mb, q, qd, qdd, tau, batch);
}
int multibody_fd_batch_host_f64(const Multibody *mb, const double *q, const double *qd, const double *tau,
                                double *qdd, int64_t batch) {
    return fd_host<double>(mb, q, qd, tau, qdd, batch);
}
int multibody_rnea_fd_batch_host_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                     const double *tau_in, double *tau, double *qdd_out, int64_t batch) {
    return idfd_host<double>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch);
}
int multibody_rnea_fd_batch_host_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                     const float *tau_in, float *tau, float *qdd_out, int64_t batch) {
    return idfd_host<float>(mb, q, qd, qdd, tau_in, tau, qdd_out, batch);
}
int multibody_rnea_batch_host_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                  float *tau, int64_t batch) {
    return rnea_host<float>(mb, q, qd, qdd, tau, batch);
}
int multibody_fd_batch_host_f32(const Multibody *mb, const float *q, const float *qd, const float *tau,
                                float *qdd, int64_t batch) {
    return fd_host<float>(mb, q, qd, tau, qdd, batch);
}

// ------------------------------------------------------------- synthetic inputs

int rb_fill_uniform_f32(float *x, int n_rows, int64_t batch, int64_t ld, const double *lo, const double *hi,
                        uint64_t seed, void *stream) {
    return fill_uniform<float>(x, n_rows, batch, ld, lo, hi, seed, stream);
}
int rb_fill_uniform_f64(double *x, int n_rows, int64_t batch, int64_t ld, const double *lo, const double *hi,
                        uint64_t seed, void *stream) {
    return fill_uniform<double>(x, n_rows, batch, ld, lo, hi, seed, stream);
}

}  // extern "C"
