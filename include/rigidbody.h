/*
 * rigidbody.h -- drop-in C ABI of khaninger/rigidbody-rs `rigidbody_bindings`.
 *
 * Same six symbols, argument meaning and result layout as the reference header
 * (rigidbody_bindings/rigidbody.h:11-16, implemented in rigidbody_bindings/src/lib.rs).
 * A C++ consumer such as rigidbody_bindings/main.cpp links librigidbody_bindings.so
 * from this repo instead of the Rust cdylib (CMakeLists.txt:11) with no source change.
 *
 * Differences, all on error paths only (the reference panics -> aborts across FFI):
 *   - a NULL handle or a failed model load returns NULL instead of aborting;
 *   - multibody_new() loads $RIGIDBODY_URDF if set, else the embedded Franka FR3
 *     model, instead of the hard-coded /home/hanikevi/... path (lib.rs:10).
 * Every query still returns a freshly allocated buffer the caller owns (the
 * reference leaks Box::into_raw results, lib.rs:28,41,55,68); it is malloc'd, so
 * free() or multibody_result_free() (rigidbody_batch.h) releases it.
 *
 * All queries compute in fp64.  One configuration per call is the reference's CPU use
 * (main.cpp:69), so these run on the calling thread with the GPU kernels' own lane bodies
 * compiled for the host (a GPU round trip per call would cost ~25x the recursion); models
 * that need model-specialised kernels (trees) launch on the GPU.  The batched entry points
 * of rigidbody_batch.h -- the actual hot path -- run on the GPU (HIP, gfx950) only.
 */
#ifndef MULTIBODY_INTERFACE_H
#define MULTIBODY_INTERFACE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct Multibody Multibody; /* opaque; reference: rigidbody_bindings/rigidbody.h:8 */

/* reference lib.rs:8-12 */
Multibody *multibody_new(void);
/* reference lib.rs:46-57: translation of the last link frame, 3 doubles */
double *multibody_fwd_kin(const Multibody *mb, const double q[7]);
/* reference lib.rs:60-70: body Jacobian of the last link, 6 x 7 column-major, rows [lin; rot] */
double *multibody_jac(const Multibody *mb, const double q[7]);
/* reference lib.rs:15-30: inverse dynamics tau, 7 doubles */
double *multibody_rnea(const Multibody *mb, const double q[7], const double dq[7], const double ddq[7]);
/* reference lib.rs:32-43: joint-space mass matrix, 7 x 7 column-major, upper triangle
 * (strictly-lower entries are exactly 0, as multibody.rs:156,166 leaves them) */
double *multibody_crba(const Multibody *mb, const double q[7]);
/* reference lib.rs:73-78: NULL-safe */
void multibody_free(Multibody *mb);

#ifdef __cplusplus
}
#endif

#endif /* MULTIBODY_INTERFACE_H */
