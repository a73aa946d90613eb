// tuning.hpp -- launch-shape knobs (host side) and resident-grid sizing.
#pragma once

namespace rbamd {

struct Tuning {
    // RNEA launch form: 1 grid-stride + register prefetch, 0 one configuration per lane,
    // -1 auto (measured on MI355X: one-per-lane for fp32 up to 8 DOF, streaming for fp64
    // and longer chains -- tools/ab_bench.py).
    int rnea_stream = -1;
    int grid_factor = 1;  // streaming grid = grid_factor x resident blocks (capped by the batch)
    int jit = 1;          // 1: model-specialised hipRTC kernels where available (jit.hpp)
    // 1: LDS-tiled 16-byte-access form of the JIT RNEA kernel when aligned.  Off: it is
    // 30% slower than the per-lane form on MI355X (block barriers serialise load/compute/
    // store; the per-lane form already runs at the pattern's copy ceiling).
    int rnea_tile = 0;
    // JIT RNEA: bit 0 non-temporal loads, bit 1 non-temporal stores (every element is
    // touched once; measured -5% fp32 / -8% fp64 kernel time).
    int rnea_nt = 3;
    // JIT forward dynamics / rollout: same bits as rnea_nt (-5% fp32 FD kernel time).
    int fd_nt = 3;
    // JIT kernels: amdgpu_waves_per_eu occupancy target; 0 compiler's choice, -1 auto
    // (4 for the fp32 rollout of chains up to 8 links: its K loop otherwise settles at
    // 129+ VGPRs, one wave per SIMD fewer; 361 vs 390 us for 16 FR3 steps).
    int jit_waves = -1;
    // Model constants pinned per use (spatial.hip.hpp mconst): 1 on, 0 off, -1 auto = the
    // rollout of chains up to 16 links (fp32 337 vs 1736 us; fp64 810 vs 995 us); off for
    // forward dynamics (fp32 29.6 vs 31.9 us once the 1/D reciprocal freed 12 VGPRs -- it
    // was 33.8 vs 35.7 the other way before; fp64 71 vs 90 us; 30-link fp32 333 vs 1331 us)
    // and for the other kinds.
    int opaque_consts = -1;
    // JIT forward dynamics: 1 = resident grid-stride form with register prefetch (aba_stream).
    int fd_stream = 0;
    // JIT fp32 RNEA / forward dynamics: 1 = two configurations per lane on packed fp32
    // (spatial.hip.hpp f2; 512 configurations per 256-lane block), 0 = one per lane,
    // -1 auto (jit_pack in jit.cpp).
    int pack = -1;
    // JIT fp64 kernels: 1 = table-assisted sincos (spatial.hip.hpp sincos_tab), 0 = the
    // pi/2-reduction minimax sincos_cw, -1 auto (on).
    int f64_tab = -1;
    // JIT RNEA of serial chains: segments of the segmented form (rnea_eval_seg); 0/1 = the
    // one-pass form, -1 auto (jit_rnea_seg in jit.cpp).
    int rnea_seg = -1;
    // JIT RNEA lane kernel (one configuration per lane): 256-configuration tiles per
    // workgroup (1, 2 or 4 -> 256 / 512 / 1024 threads).
    int rnea_tiles = 1;
    // JIT ABA / CRBA: rotate symmetric inertia blocks as R_p (Rz S Rz^T) R_p^T with the double
    // angle (artinertia.hip.hpp to_parent_split); 0 = the folded E S E^T; -1 auto = on when
    // every joint frame R_p is a signed permutation.
    int split_rot = -1;
    // Free experiment selector, emitted as RB_VARIANT into every JIT source (A/B only).
    int jit_variant = 0;
};

// Process-wide knobs, initialised from RB_RNEA_STREAM / RB_GRID_FACTOR / RB_JIT, adjustable through
// rb_set_tuning() (used by the A/B benchmarks; not needed for normal use).
Tuning &tuning();

// Blocks for a streaming launch of `kfn`: factor x (resident blocks per CU x CUs) on the
// current device, never more than `full` (one block per 256 configurations).  Cached per
// (device, kernel).
unsigned stream_grid(const void *kfn, int block, unsigned full, int factor);

// RNEA launch form.  Measured (tools/ab_bench.py): for the precompiled
// generic kernels the streaming form wins for fp64 and chains longer than 8 links; the
// model-specialised (JIT) kernels are lighter and the one-per-lane form wins everywhere.
inline bool rnea_use_stream(bool f64, int n, bool jit) {
    const int v = tuning().rnea_stream;
    if (v >= 0) return v != 0;
    return jit ? false : (f64 || n > 8);
}

}  // namespace rbamd
