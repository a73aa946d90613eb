// kernels.hpp -- host-side launch entry points of the batched kernels.
//
// Design: one lane = one configuration.  Joint states are SoA
// (x[j*ld + b]) so every per-joint load/store of a wavefront is one coalesced
// 256 B (fp32) / 512 B (fp64) transaction -- or, with `tiled`, the tiled layout
// x[((b / 256) * rows + j) * 256 + b % 256] (rows = n for joint arrays), which keeps a
// 256-configuration tile of every row in one contiguous block (20-25% closer to the HBM
// copy ceiling on the RNEA pattern).  The chain recursion runs inside the lane,
// fully unrolled over the compile-time DOF N (dofs.hpp), so every per-link quantity
// (forces, articulated inertias, sin/cos) lives in VGPRs; the model constants (layout.hpp)
// are staged in LDS per block by the generic kernels and are compile-time immediates in the
// model-specialised ones (jit.cpp).  No MFMA: there is no dense contraction on this path.
//
// Kernel families (reference function each one batches):
//   rnea.hip        Multibody::rnea       multibody.rs:111-153
//   aba.hip         forward dynamics, defined as sym(H)^-1 (tau - rnea(q,qd,0)) with H
//                   from Multibody::crba (multibody.rs:155-174); computed by the
//                   Articulated-Body Algorithm (Featherstone Table 7.1)
//   crba.hip        Multibody::crba       multibody.rs:155-174 (upper triangle, lower = 0)
//   kinematics.hip  Multibody::fwd_kin / jac  multibody.rs:87-108; synthetic input fill
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rbamd {

int supported_dofs(int *out, int cap);
bool dof_supported(int n);

template <typename T>
hipError_t launch_rnea(int n, const T *mdl, const T *q, const T *qd, const T *qdd, T *tau,
                       uint32_t B, int64_t ld, hipStream_t s, bool fast, bool tiled);
template <typename T>
hipError_t launch_aba(int n, const T *mdl, const T *q, const T *qd, const T *tau, T *qdd,
                      uint32_t B, int64_t ld, hipStream_t s, bool fast, bool tiled);
// SoA [rows][ld] <-> tiled [ceil(B/256)][rows][256] (tail lanes of the last tile written as 0).
template <typename T>
hipError_t launch_to_tiled(const T *src, int64_t ld, T *dst, int rows, uint32_t B, hipStream_t s);
template <typename T>
hipError_t launch_from_tiled(const T *src, T *dst, int64_t ld, int rows, uint32_t B, hipStream_t s);
template <typename T>
hipError_t launch_rollout(int n, const T *mdl, T *q, T *qd, const T *tau_seq, T dt, int K, T *traj, uint32_t B,
                          int64_t ld, hipStream_t s, bool fast);
template <typename T>
hipError_t launch_crba(int n, const T *mdl, const T *q, T *H, uint32_t B, int64_t ld,
                       hipStream_t s, bool tiled = false);
template <typename T>
hipError_t launch_fwd_kin(int n, const T *mdl, const T *q, T *pos, uint32_t B, int64_t ld,
                          hipStream_t s, bool fast, bool tiled = false);
template <typename T>
hipError_t launch_jac(int n, const T *mdl, const T *q, T *J, uint32_t B, int64_t ld,
                      hipStream_t s, bool fast, bool tiled = false);
template <typename T>
hipError_t launch_fill_uniform(T *x, int rows, uint32_t B, int64_t ld, const double *lohi_dev,
                               uint64_t seed, hipStream_t s);

}  // namespace rbamd
