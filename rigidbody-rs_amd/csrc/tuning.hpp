// tuning.hpp -- launch-shape knobs (host side) and resident-grid sizing.
//
// Production knobs (rb_set_tuning accepts these always): `jit`, `pack`, `rnea_stream`,
// `single_gpu`, `fd_form`, `rnea_park`, `rnea_rev`.
// Everything else is an A/B experiment selector: rb_set_tuning accepts it only when the
// process runs with RB_EXPERIMENTAL=1 (tools/ab_bench.py, tools/small_batch.py), so a normal
// caller cannot multiply the hipRTC kernel variants (jit.cpp cache key) or the test matrix.
#pragma once

#include <atomic>

namespace rbamd {

// Every knob is an atomic int: rb_set_tuning may run while other threads launch (a launch
// reads each knob once; a concurrent change applies to the launches that read it after).
struct Tuning {
    // ---- production
    std::atomic<int> jit{1};  // 1: model-specialised hipRTC kernels where available (jit.hpp)
    // JIT fp32 forward dynamics / rollout lane form: 2 = two configurations per lane on packed
    // fp32 (spatial.hip.hpp f2; 512 configurations per 256-lane block), 1 = one per lane,
    // 4 = bias / mass-matrix split over a pair of packed waves, 5 = that split one per lane;
    // RNEA: 3 = two configurations per lane one after the other, 1 = one per lane;
    // -1 auto (capi.cpp jit_rnea / jit_fd / launch_rollout_any by batch size and layout,
    // jit.cpp jit_pack).
    std::atomic<int> pack{-1};
    // Precompiled (generic) RNEA launch form: 1 grid-stride + register prefetch, 0 one
    // configuration per lane, -1 auto (streaming for fp64 and chains longer than 8 links,
    // where it measured 7-9% faster -- DESIGN.md §4).  The model-specialised kernels are
    // always one configuration per lane.
    std::atomic<int> rnea_stream{-1};
    // Single-configuration ABI (multibody_rnea / _crba / _fwd_kin / _jac): 0 = on the calling
    // host thread with the lane bodies compiled for the host (host_eval.cpp) where the model
    // allows it, 1 = always a GPU launch (H2D, kernel, D2H, sync).
    std::atomic<int> single_gpu{0};
    // Forward dynamics algorithm of the model-specialised kernels: 1 = Articulated-Body
    // Algorithm (aba_body.hip.hpp), 2 = mass-matrix method (fdh_body.hip.hpp: bias torques by
    // RNEA, H by CRBA, L D L^T solve -- the oracle's own definition), -1 auto (jit.cpp
    // jit_fd_form: mass matrix for serial chains up to 12 links, rollouts up to 8).
    std::atomic<int> fd_form{-1};
    // JIT fp32 RNEA of long serial chains: the first `rnea_park` links' forces parked in LDS and
    // (cos, sin) re-evaluated from reloaded q (rnea_body.hip.hpp rnea_lane_park), 3 waves/SIMD
    // instead of 2; 0 = off, -1 auto (8 for chains of 20+ links: 30-link 2^20 91.0 vs 103.4 us,
    // bit-identical).
    std::atomic<int> rnea_park{-1};
    // JIT fp64 RNEA of serial chains longer than 8 links: the reversed-sweep form
    // (rnea_body.hip.hpp rnea_lane_rev: the backward sweep recovers each parent's kinematics by
    // inverting the forward step, no per-link storage, 2-3 waves/SIMD); 0 = off, 1 = on,
    // -1 auto = on (2^20 tiled: 12 links 81.8 vs 87.2 us, 16 links 114.7 vs 112.1, 30 links 234
    // vs 321).
    std::atomic<int> rnea_rev{-1};

    // ---- experimental (RB_EXPERIMENTAL=1)
    std::atomic<int> grid_factor{1};  // streaming grid = grid_factor x resident blocks (capped by the batch)
    // JIT RNEA: bit 0 non-temporal loads, bit 1 non-temporal stores (every element is
    // touched once; fp64 FR3 2^20 tiled 39.9 vs 42.7 us without, 30-DOF 91.4 vs 98.6, 65536
    // fp32 3.46 vs 3.89); -1 auto = 3, except 0 for the fp32 RNEA of chains up to 8 links at
    // batches >= 2^19 on the tiled layout (FR3 2^20: 22.4 vs 25.2 us, steady where nt=3 swings
    // 20-25; SoA rows keep 3: 24.3 vs 24.9; the 30-link chain 99.9 vs 91.3 and the 14-DOF tree
    // 44.2 vs 41.2 keep 3) -- capi.cpp jit_rnea.
    std::atomic<int> rnea_nt{-1};
    // JIT forward dynamics / rollout: same bits as rnea_nt (-5% fp32 FD kernel time).
    std::atomic<int> fd_nt{3};
    // JIT kernels: amdgpu_waves_per_eu occupancy target; 0 compiler's choice, -1 auto:
    // 4 for the fp32 rollout of chains up to 8 links (its K loop otherwise settles at 129+
    // VGPRs, one wave per SIMD fewer; 361 vs 390 us for 16 FR3 steps), for the
    // paired fp32 mass-matrix FD and for the fp64 mass-matrix rollout (jit.cpp jit_source);
    // 2 where a kernel built without one lands just past 256 registers (jit.cpp jit_compile,
    // the occupancy cliff).  Any value >= 0 disables the automatic ones.
    std::atomic<int> jit_waves{-1};
    // Model constants pinned per use (spatial.hip.hpp mconst): 1 on, 0 off, -1 auto = the
    // rollout of chains up to 16 links (fp32 337 vs 1736 us; fp64 810 vs 995 us); off for
    // forward dynamics (fp32 29.6 vs 31.9 us; fp64 71 vs 90 us; 30-link fp32 333 vs 1331 us)
    // and for the other kinds.
    std::atomic<int> opaque_consts{-1};
    // JIT fp64 kernels: 1 = table-assisted sincos (spatial.hip.hpp sincos_tab), 0 = the
    // pi/2-reduction minimax sincos_cw, -1 auto (on).
    std::atomic<int> f64_tab{-1};
    // JIT ABA / CRBA: rotate symmetric inertia blocks as R_p (Rz S Rz^T) R_p^T with the double
    // angle (artinertia.hip.hpp to_parent_split); 0 = the folded E S E^T; -1 auto = on when
    // every joint frame R_p is a signed permutation.
    std::atomic<int> split_rot{-1};
    // Free experiment selector, emitted as RB_VARIANT into every JIT source (A/B only).
    std::atomic<int> jit_variant{0};
    // Sequential-pair RNEA (pack 3): the last `seq_tail` percent of a launch's 256-configuration
    // tiles run one configuration per lane, so the blocks dispatched last carry half the
    // dependent chain (the launch's compute tail after its last rows land).  0 = all pairs,
    // -1 auto: 75 for the tiled layout (FR3 fp64 2^20: 40.5 vs 41.8 us), 0 for SoA (43.6-45.9 vs
    // 42.9 us), DESIGN.md §4.
    std::atomic<int> seq_tail{-1};
    // Batched fwd_kin / jac of serial revolute chains: 1 = the model-specialised hipRTC kernels
    // (tree_body.hip.hpp fwd_kin_tree / jac_tree with the chain's topology), 0 = the precompiled
    // kernels (kinematics.hip), -1 auto (the hipRTC kernels: fwd_kin fp64 18.2 vs 26.4 us at 2^20).
    std::atomic<int> kin_jit{-1};
    // JIT CRBA / fwd_kin / jac: same bits as rnea_nt; -1 auto = 2 for CRBA and jac
    // (non-temporal stores: the outputs are written once; FR3 2^20 fp64 CRBA 84.7 vs 102.9 us,
    // jac 70.3 vs 89.3, fp32 CRBA 40.5 vs 46.2 -- at the no-math probe's 5.9 TB/s for these row
    // shapes), 3 for fwd_kin (16.4 vs 17.2 with stores only, 18.3 with neither).
    std::atomic<int> kin_nt{-1};
    // JIT kernels: the first `kernarg_preload` dwords of the kernel arguments arrive in SGPRs
    // with the dispatch (-amdgpu-kernarg-preload-count; 14 = every user SGPR the kernarg pointer
    // leaves) instead of by scalar loads at entry -- the code object keeps a 256-byte prologue
    // that loads them for firmware without preload.  0 = off.  Interleaved A/B, HIP graph, two
    // boxes (profiles/r06/ab/ab_*_preload.log): RNEA fp32 65536 3.58-3.60 vs 3.62-3.65 us, FD fp32
    // 65536 4.11-4.13 vs 4.16-4.18; the fused fp64 2^17 shard and the headline within noise.
    std::atomic<int> kernarg_preload{14};
};

// Process-wide knobs, initialised from RB_JIT / RB_PACK / RB_RNEA_STREAM (and, with
// RB_EXPERIMENTAL=1, the experimental RB_* variables), adjustable through rb_set_tuning().
Tuning &tuning();

// Whether RB_EXPERIMENTAL=1 is set (experimental knobs writable).
bool tuning_experimental();

// Sets `key`; returns 0, 1 (unknown key) or 2 (experimental key without RB_EXPERIMENTAL=1).
int tuning_set(const char *key, int value);

// Advanced twice by every successful tuning_set (odd while the write is in progress, even
// otherwise): per-launch caches keyed on the tuning state (capi.cpp jit_get's fast path)
// compare it instead of rebuilding their string keys.
unsigned tuning_generation();
// The current generation once no rb_set_tuning write is in progress (an even sequence count).
unsigned tuning_generation_stable();

// Blocks for a streaming launch of `kfn`: factor x (resident blocks per CU x CUs) on the
// current device, never more than `full` (one block per 256 configurations).  Cached per
// (device, kernel).
unsigned stream_grid(const void *kfn, int block, unsigned full, int factor);

// RNEA launch form of the precompiled kernels (the JIT kernels are one per lane).
inline bool rnea_use_stream(bool f64, int n) {
    const int v = tuning().rnea_stream;
    if (v >= 0) return v != 0;
    return f64 || n > 8;
}

}  // namespace rbamd
