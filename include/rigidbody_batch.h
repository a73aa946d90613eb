/*
 * rigidbody_batch.h -- batched GPU extension of the rigidbody_bindings C ABI.
 *
 * The reference exposes one configuration per call (rigidbody_bindings/src/lib.rs:15-70).
 * These entry points evaluate B configurations per call on one MI355X (gfx950) with
 * hand-written HIP kernels.  They replace, for a batch, a loop of the reference calls:
 *
 *   multibody_rnea_batch_*     <- multibody_rnea      (lib.rs:15-30, multibody.rs:111-153)
 *   multibody_fd_batch_*       <- no reference entry point: forward dynamics defined as
 *                                 qdd = sym(H)^-1 (tau - rnea(q,qd,0)) with H from
 *                                 multibody_crba (multibody.rs:155-174) (SURVEY.md §8(a)
 *                                 A10), computed by exactly that definition fused per
 *                                 configuration (RNEA bias + CRBA + L D L^T) for serial chains
 *                                 up to 12 links, by the Articulated-Body Algorithm otherwise
 *                                 (rb_set_tuning "fd_form")
 *   multibody_rnea_fd_batch_*  <- both of the above on one (q, qd): tau = rnea(q, qd, qdd) and
 *                                 qdd' = fd(q, qd, tau_in) in one launch (SURVEY.md §8(d)
 *                                 config 4's RNEA + forward-dynamics pair)
 *   multibody_rollout_batch_*  <- K fused forward-dynamics + semi-implicit Euler steps
 *                                 (MPC shooting)
 *   multibody_crba_batch_*     <- multibody_crba      (lib.rs:32-43)
 *   multibody_fwd_kin_batch_*  <- multibody_fwd_kin   (lib.rs:46-57)
 *   multibody_jac_batch_*      <- multibody_jac       (lib.rs:60-70)
 *
 * Layout: structure of arrays.  Joint j of configuration b lives at x[j * ld + b]
 * (ld >= batch, the leading dimension).  Matrix outputs store element e of each
 * configuration at out[e * ld + b], with e following the single-call ABI's
 * column-major order (crba: e = row + n*col; jac: e = row + 6*col; fwd_kin: e = 0..2).
 *
 * Batch size: any batch >= 0 (0 = nothing to do); one kernel launch covers at most 2^28
 * configurations (lane byte offsets are 32-bit), larger batches are split into consecutive
 * launches on the same stream (tests/test_gpu_limits.py: 2^28 + 257).  rb_fill_uniform_*
 * alone takes at most 2^28 columns per call.
 *
 * Pointers: the plain entry points take DEVICE pointers (hipMalloc'd memory on the
 * current HIP device) and enqueue asynchronously on `stream` (a hipStream_t; NULL =
 * the null stream).  The *_host variants take host pointers and block until done.
 *
 * Return value: RB_OK (0) or an rb_status error code; rb_last_error() gives a
 * thread-local message.  No entry point aborts the process.
 *
 * Reentrancy: a Multibody is immutable after construction; calls on one handle
 * from several threads are safe (device model constants are uploaded once per
 * device under a lock; the single-config ABI uses thread-local staging).
 *
 * Input domain.  The reference evaluates any f64 joint angle exactly (libm sin/cos in
 * UnitQuaternion::from_scaled_axis, joint.rs:48-50) and lets NaN / Inf flow through its
 * arithmetic.  The batched kernels are exact (at the |q| <= pi tolerances of the tests) for
 *   every input finite (|x| < 2^1017 in fp64) and every revolute angle |q_j| < 2^41 rad
 *   (fp64) / 2^22 rad (fp32)
 * -- each sincos reduces the angle exactly over that range (spatial.hip.hpp; tested in every
 * kernel form at |q| from 10 rad to just below the bound -- fp64 1e9, 1e12, 2^40, 2^41 - 4 --
 * and at exactly the bound, tests/test_gpu_domain.py).  A configuration outside it -- a NaN or
 * +-Inf in any of its inputs, or an angle past the bound -- gets NaN in EVERY output (CRBA:
 * every upper-triangle entry; the strictly-lower entries stay the ABI's exact zeros), in
 * every kernel form; the other configurations of the batch, including the other half of a
 * paired lane, are unaffected.  Rollouts check the state and tau_k every step: a trajectory
 * is NaN from the step its input went bad.  (The reference yields NaN exactly in the outputs
 * that depend on the bad input -- every torque of rnea; H and J keep the entries that do
 * not; these kernels poison the whole configuration.)  The single-configuration ABI
 * (rigidbody.h) computes every finite angle exactly, as the reference, and returns NaN
 * outputs for NaN / Inf inputs.
 *
 * Accuracy (tests/test_gpu_parity.py, test_gpu_domain.py, against the fp64 oracle).  fp64 RNEA,
 * CRBA, fwd_kin, jac: |d| <= 1e-9 (1 + |ref|) element-wise.  fp64 forward dynamics is a
 * backward-stable solve (L D L^T, or the ABA): with H_s = sym(H), C = rnea(q, qd, 0),
 *   |H_s qdd - (tau - C)|_inf <= n eps64 (|H_s|_inf |qdd|_inf + |tau - C|_inf)
 *   |qdd - qdd_exact|_inf     <= 4 eps64 cond(H_s) (1 + |qdd_exact|_inf)
 * -- at any conditioning (tested to cond(H) ~ 1e14, a floating base within 1e-6 rad of its pitch
 * singularity); for cond(H) <= ~1e4 (FR3 over its limits) that is a torque residual
 * |rnea(q, qd, qdd) - tau| <= 1e-8 (1 + |tau|).  fp32: RNEA 1e-4 (1 + |tau|) (chains past ~20
 * links column-norm-wise: root torques lose digits to cancellation in any fp32 evaluation),
 * forward dynamics |rnea64(q, qd, qdd32) - tau| <= 24 eps32 (1 + |tau| + |H_s| |qdd32|).
 */
#ifndef RIGIDBODY_BATCH_H
#define RIGIDBODY_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "rigidbody.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    RB_OK = 0,
    RB_ERR_NULL = 1,        /* NULL handle or pointer */
    RB_ERR_ARG = 2,         /* bad size / leading dimension / buffer length */
    RB_ERR_HIP = 3,         /* HIP runtime error (message in rb_last_error) */
    RB_ERR_URDF = 4,        /* URDF could not be read or parsed */
    RB_ERR_DOF = 5,         /* DOF outside the compiled kernel set */
    RB_ERR_UNSUPPORTED = 6, /* model feature outside the reference's semantics */
    RB_ERR_NUMERIC = 7      /* singular articulated inertia in FD */
} rb_status;

/* ---- model construction ------------------------------------------------------- */
/* Multibody::from_urdf (multibody.rs:65-77) on a file / an in-memory string.  Any
 * number of revolute joints for which a kernel is compiled (multibody_supported_dofs);
 * with RB_MODEL_URDF_TREE, trees / prismatic joints of up to 64 DOF (hipRTC kernels). */
Multibody *multibody_new_from_urdf(const char *path);
Multibody *multibody_new_from_urdf_string(const char *xml, size_t len);

/* Model-reading flags, beyond the reference.  0 = the reference's
 * reading: top-level joints/links paired by index, fixed joints dropped, z axes only
 * (multibody.rs:65-77, 130-138).
 *   RB_MODEL_GENERAL_AXES: any revolute axis, motion subspace S = (axis, 0).  Identical
 *     results for z-axis chains.  fwd_kin/jac stay in the URDF link frames.
 *   RB_MODEL_URDF_TREE: follow joint parent/child names from the root link; fixed joints
 *     are merged (child inertia into the parent body, origin into the next joint); the
 *     inertial-origin rpy is honoured; kinematic trees (links numbered depth-first, parent
 *     index < child index, multibody_topology) with revolute / continuous / prismatic
 *     joints; mimic joints are rejected (RB_ERR_URDF).  Trees and prismatic joints run only
 *     on model-specialised (hipRTC) kernels; fwd_kin / jac then follow the last link's
 *     ancestor path (other Jacobian columns zero), CRBA keeps the upper-triangle layout
 *     with exact zeros for unrelated joint pairs.
 *   RB_MODEL_FLOATING_BASE: a free-floating root body: six massless virtual joints first --
 *     prismatic along world x, y, z, then revolute about z, y, x (yaw / pitch / roll; the
 *     root orientation is Rz Ry Rx, singular at pitch = +-pi/2).  Implies the two flags
 *     above.  Gravity stays the reference's +9.81 base acceleration (multibody.rs:117-120),
 *     so a free fall reads qdd = (0, 0, -9.81, 0, ...). */
enum { RB_MODEL_GENERAL_AXES = 1, RB_MODEL_URDF_TREE = 2, RB_MODEL_FLOATING_BASE = 4 };
Multibody *multibody_new_from_urdf_ex(const char *path, unsigned flags);
Multibody *multibody_new_from_urdf_string_ex(const char *xml, size_t len, unsigned flags);
unsigned multibody_flags(const Multibody *mb);
/* Packed fp64 model (bit-exact), for broadcasting one model to every rank (RCCL). */
int64_t multibody_blob_size(const Multibody *mb);                 /* in doubles */
int multibody_export_blob(const Multibody *mb, double *out, int64_t len);
Multibody *multibody_new_from_blob(const double *blob, int64_t len);

int multibody_dof(const Multibody *mb);
/* Total moving mass (sum of link masses). */
double multibody_total_mass(const Multibody *mb);
/* Joint limits parsed from the URDF (NaN where absent); arrays of multibody_dof. */
int multibody_limits(const Multibody *mb, double *lower, double *upper,
                     double *velocity, double *effort);
/* Writes up to `cap` DOF values the kernels are compiled for; returns their count. */
int multibody_supported_dofs(int *out, int cap);
/* Per link: parent link index (-1 = base; the reference's chain has i - 1) and joint type
 * (0 revolute, 1 prismatic).  Either array may be NULL. */
int multibody_topology(const Multibody *mb, int *parent, int *joint_type);

/* Uploads the model constants to the current HIP device now (otherwise done lazily on
 * the first batched call); call before capturing batched calls into a hipGraph. */
int multibody_upload(const Multibody *mb);

/* Which kernel a launch of `batch` configurations (tiled != 0: the *_tiled entry points)
 * runs for this model on the current device; kind 0 = rnea, 1 = fd, 2 = crba, 3 = rollout,
 * 4 = fwd_kin, 5 = jac, 6 = rnea_fd (multibody_rnea_fd_batch_*).  1 = model-specialised kernel
 * compiled at first use by hipRTC (this call compiles exactly the form such a launch takes), 0 =
 * precompiled generic kernel (also when hipRTC failed; rb_last_error() holds the log -- a tree
 * model's calls then fail with RB_ERR_UNSUPPORTED; kind 6: the model has no fused kernel and
 * runs the rnea then the fd kernel).  multibody_kernel_path = a 2^20-configuration SoA launch. */
int multibody_kernel_path_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled);
int multibody_kernel_path(const Multibody *mb, int kind, int f64);
int multibody_rnea_kernel_path(const Multibody *mb, int f64);
/* The launch form of that kernel (same resolution, compiles it if needed): 0 = precompiled
 * generic kernel, else the model-specialised kernel's configurations-per-lane form -- 1 one per
 * lane, 2 two per lane on packed fp32, 3 two per lane one after the other (the fp64 RNEA from
 * 2^19 configurations, and the fp32 RNEA of chains up to 8 links on the tiled layout from 2^19,
 * compiled there with ordinary instead of non-temporal loads / stores), 4 / 5 the bias /
 * mass-matrix wave split packed / one per lane (fp32 mass-matrix forward dynamics and rollouts
 * up to 2^17 configurations).  Negative = -status on a bad argument. */
int multibody_kernel_form_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled);
/* Where the reference's single-configuration queries (rigidbody.h: rnea, crba, fwd_kin,
 * jac) run for this model: 0 = on the calling host thread (the GPU lane bodies compiled for
 * the host; serial revolute chains of a precompiled DOF on an FMA3/AVX2 CPU), 1 = one GPU
 * launch per call (trees / prismatic joints, or rb_set_tuning("single_gpu", 1)). */
int multibody_single_config_path(const Multibody *mb);
/* The generated source of the model-specialised kernel a launch of `batch` configurations
 * (tiled != 0: the *_tiled entry points) runs -- the same form, tail and load / store policy
 * multibody_kernel_form_ex reports, and the occupancy target the occupancy-cliff rebuild adds
 * (the source is hipRTC-compiled for gfx950 to decide it, no device needed); returns its length;
 * copies at most cap-1 bytes + NUL into buf when buf != NULL.  multibody_jit_source = a
 * 2^20-configuration SoA launch. */
int multibody_jit_source_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled, char *buf,
                            int64_t cap);
int multibody_jit_source(const Multibody *mb, int kind, int f64, char *buf, int64_t cap);
/* hipRTC-compiles that kernel for `arch` (NULL = "gfx950") without a device; returns
 * the code-object size, or minus an rb_status code (log in rb_last_error()). */
int64_t multibody_jit_compile_ex(const Multibody *mb, int kind, int f64, int64_t batch, int tiled,
                                 const char *arch);
int64_t multibody_jit_compile(const Multibody *mb, int kind, int f64, const char *arch);

void multibody_result_free(double *p);
const char *rb_last_error(void);
const char *rb_version(void);
/* Launch-shape knobs for A/B measurements (keys and defaults: INTEGRATION.md "Knobs",
 * rigidbody-rs_amd/csrc/tuning.hpp); defaults are the tuned values.  Process-wide. */
int rb_set_tuning(const char *key, int value);

/* ---- batched device-pointer entry points (asynchronous on `stream`) ------------ */
int multibody_rnea_batch_f32(const Multibody *mb, const float *q, const float *qd,
                             const float *qdd, float *tau, int64_t batch, int64_t ld,
                             void *stream);
int multibody_rnea_batch_f64(const Multibody *mb, const double *q, const double *qd,
                             const double *qdd, double *tau, int64_t batch, int64_t ld,
                             void *stream);
int multibody_fd_batch_f32(const Multibody *mb, const float *q, const float *qd,
                           const float *tau, float *qdd, int64_t batch, int64_t ld,
                           void *stream);
int multibody_fd_batch_f64(const Multibody *mb, const double *q, const double *qd,
                           const double *tau, double *qdd, int64_t batch, int64_t ld,
                           void *stream);
/* Tiled layout (same computation): every array is [ceil(batch/256)][rows][256], element
 * (row j, configuration b) at ((b / 256) * rows + j) * 256 + b % 256, rows = n -- each
 * 256-configuration tile of all joints contiguous.  Measured on MI355X (bench.py layout_ab_*
 * lines, interleaved in one process, driver runs): fp64 RNEA 3-6% faster than SoA rows, fp32
 * RNEA ~5% faster, fp64 FD equal -- use it when the data is produced tiled, not by converting.  Allocate
 * whole tiles; lanes past `batch` in the last tile are neither read nor written. */
int multibody_rnea_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                   float *tau, int64_t batch, void *stream);
int multibody_rnea_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                   double *tau, int64_t batch, void *stream);
int multibody_fd_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *tau,
                                 float *qdd, int64_t batch, void *stream);
int multibody_fd_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *tau,
                                 double *qdd, int64_t batch, void *stream);
/* Inverse and forward dynamics of the same (q, qd) in one launch:
 *   tau     = rnea(q, qd, qdd)                   (multibody_rnea_batch_*, multibody.rs:111-153)
 *   qdd_out = sym(H)^-1 (tau_in - rnea(q, qd, 0)) (multibody_fd_batch_*)
 * For models on the mass-matrix forward dynamics (serial revolute chains up to 12 links) one
 * fused kernel evaluates both from one set of factors: the bias torques C = rnea(q, qd, 0), H
 * (multibody.rs:155-174) and its L D L^T, with tau = C + sym(H) qdd -- the RNEA is affine in qdd
 * with slope H -- so q and qd are read once: 6 n s bytes per configuration against 8 n s for
 * the two calls, and one launch.  tau agrees with multibody_rnea_batch_* to rounding (not bit
 * for bit: a different order of the same sums; tested against the oracle at 1e-9 scaled in
 * fp64), qdd_out with multibody_fd_batch_* bit for bit.  Other models run the two kernels
 * back to back on `stream`.  Input domain as above, per output: tau is NaN for a configuration
 * whose q, qd or qdd is out of the domain, qdd_out for one whose q, qd or tau_in is.  Outputs
 * must not overlap the inputs or each other (an output passed as an input, e.g. tau_in as tau,
 * is refused with RB_ERR_ARG). */
int multibody_rnea_fd_batch_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                const float *tau_in, float *tau, float *qdd_out, int64_t batch, int64_t ld,
                                void *stream);
int multibody_rnea_fd_batch_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                const double *tau_in, double *tau, double *qdd_out, int64_t batch, int64_t ld,
                                void *stream);
int multibody_rnea_fd_batch_tiled_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                      const float *tau_in, float *tau, float *qdd_out, int64_t batch, void *stream);
int multibody_rnea_fd_batch_tiled_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                      const double *tau_in, double *tau, double *qdd_out, int64_t batch,
                                      void *stream);
/* Blocking host-pointer form ([n][batch] host arrays in and out), as the *_batch_host_* below. */
int multibody_rnea_fd_batch_host_f64(const Multibody *mb, const double *q, const double *qd, const double *qdd,
                                     const double *tau_in, double *tau, double *qdd_out, int64_t batch);
int multibody_rnea_fd_batch_host_f32(const Multibody *mb, const float *q, const float *qd, const float *qdd,
                                     const float *tau_in, float *tau, float *qdd_out, int64_t batch);
/* SoA [rows][ld] <-> tiled [ceil(batch/256)][rows][256] (to_tiled zero-fills the tail lanes). */
int rb_to_tiled_f32(const float *src, int64_t ld, float *dst, int rows, int64_t batch, void *stream);
int rb_to_tiled_f64(const double *src, int64_t ld, double *dst, int rows, int64_t batch, void *stream);
int rb_from_tiled_f32(const float *src, float *dst, int64_t ld, int rows, int64_t batch, void *stream);
int rb_from_tiled_f64(const double *src, double *dst, int64_t ld, int rows, int64_t batch, void *stream);

/* Fused rollout for MPC shooting: K steps of semi-implicit Euler on the forward dynamics
 * above (the same algorithm the fd entry points use), qd += dt * qdd(q, qd, tau_k); q += dt * qd, the state
 * kept on chip between steps (LDS for fp32 chains up to 16 links, registers otherwise; below
 * 2^17 fp32 configurations each step is split over a pair of waves sharing the state in LDS).  q and qd
 * ([n][ld]) are read and overwritten with the final state; tau_seq is [K][n][ld] (step k,
 * joint j, config b at (k*n + j)*ld + b); traj (same shape, may be NULL) receives q after
 * every step. */
int multibody_rollout_batch_f32(const Multibody *mb, float *q, float *qd, const float *tau_seq,
                                double dt, int K, float *traj, int64_t batch, int64_t ld,
                                void *stream);
int multibody_rollout_batch_f64(const Multibody *mb, double *q, double *qd, const double *tau_seq,
                                double dt, int K, double *traj, int64_t batch, int64_t ld,
                                void *stream);
int multibody_crba_batch_f32(const Multibody *mb, const float *q, float *H,
                             int64_t batch, int64_t ld, void *stream);
int multibody_crba_batch_f64(const Multibody *mb, const double *q, double *H,
                             int64_t batch, int64_t ld, void *stream);
int multibody_fwd_kin_batch_f64(const Multibody *mb, const double *q, double *pos,
                                int64_t batch, int64_t ld, void *stream);
int multibody_jac_batch_f64(const Multibody *mb, const double *q, double *J,
                            int64_t batch, int64_t ld, void *stream);
/* The same in fp32 (the reference computes them in fp64, lib.rs:46-70; fp32 for callers that
 * keep their batch in fp32). */
int multibody_fwd_kin_batch_f32(const Multibody *mb, const float *q, float *pos,
                                int64_t batch, int64_t ld, void *stream);
int multibody_jac_batch_f32(const Multibody *mb, const float *q, float *J,
                            int64_t batch, int64_t ld, void *stream);
/* The q-only queries on the tiled layout: q is [ceil(batch/256)][n][256], the output
 * [ceil(batch/256)][rows][256] with rows = n*n (crba), 6n (jac), 3 (fwd_kin), elements in the
 * same order as the SoA rows above.  Bit-identical to the SoA forms. */
int multibody_crba_batch_tiled_f32(const Multibody *mb, const float *q, float *H, int64_t batch, void *stream);
int multibody_crba_batch_tiled_f64(const Multibody *mb, const double *q, double *H, int64_t batch, void *stream);
int multibody_fwd_kin_batch_tiled_f32(const Multibody *mb, const float *q, float *pos, int64_t batch,
                                      void *stream);
int multibody_fwd_kin_batch_tiled_f64(const Multibody *mb, const double *q, double *pos, int64_t batch,
                                      void *stream);
int multibody_jac_batch_tiled_f32(const Multibody *mb, const float *q, float *J, int64_t batch, void *stream);
int multibody_jac_batch_tiled_f64(const Multibody *mb, const double *q, double *J, int64_t batch, void *stream);

/* ---- batched host-pointer entry points (blocking) ------------------------------ */
int multibody_rnea_batch_host_f64(const Multibody *mb, const double *q, const double *qd,
                                  const double *qdd, double *tau, int64_t batch);
int multibody_fd_batch_host_f64(const Multibody *mb, const double *q, const double *qd,
                                const double *tau, double *qdd, int64_t batch);
int multibody_rnea_batch_host_f32(const Multibody *mb, const float *q, const float *qd,
                                  const float *qdd, float *tau, int64_t batch);
int multibody_fd_batch_host_f32(const Multibody *mb, const float *q, const float *qd,
                                const float *tau, float *qdd, int64_t batch);

/* ---- synthetic inputs, generated on device ------------------------------------- */
/* x[j*ld + b] = lo[j] + (hi[j]-lo[j]) * u(seed, j, b), u = splitmix64 -> [0,1) with
 * 53-bit (f64) / 24-bit (f32) mantissa; lo/hi are host arrays of n_rows. */
int rb_fill_uniform_f32(float *x, int n_rows, int64_t batch, int64_t ld, const double *lo,
                        const double *hi, uint64_t seed, void *stream);
int rb_fill_uniform_f64(double *x, int n_rows, int64_t batch, int64_t ld, const double *lo,
                        const double *hi, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* RIGIDBODY_BATCH_H */
