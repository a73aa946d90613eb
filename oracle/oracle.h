/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * fp64 CPU restatement of khaninger/rigidbody-rs (reference @ 2025-02-24) for the
 * RNEA / CRBA / fwd_kin / jac hot path, plus the forward-dynamics *definition*
 * qdd = sym(H)^-1 (tau - rnea(q, qd, 0)) (the reference has no ABA).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product library (rigidbody-rs_amd/csrc) never links or calls it.
 *
 * Parity status: the reference (Rust, nightly, nalgebra 0.33.2 / xurdf 0.2.5) cannot be
 * built here (no cargo/rustc, no network), and the reference's own tests hold no
 * RNEA/CRBA outputs.  This restatement is pinned by (1) the reference's own
 * transform known-answer tests (spatial.rs:283-382), restated in
 * tests/test_oracle.py, (2) an independent 6x6 Featherstone-matrix formulation
 * (oracle/featherstone6.py, spatial.rs:32-85 + inertia.rs:53-70 forms) to <=1e-12,
 * and (3) physics invariants (SURVEY §8(c) i-vi).
 */
#ifndef RB_ORACLE_H
#define RB_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_DOF 64

/* Mirrors `Multibody([RevoluteJoint; 7])` (multibody.rs:32) generalised to n links.
 * Each RevoluteJoint {axis, parent: Isometry3, body: Inertia} (joint.rs:26-31,
 * inertia.rs:12-18).  Quaternions are stored in nalgebra coordinate order (i, j, k, w). */
typedef struct {
    int n;
    double axis[ORACLE_MAX_DOF][3];
    double pq[ORACLE_MAX_DOF][4];   /* parent rotation, unit quaternion (i,j,k,w) */
    double pt[ORACLE_MAX_DOF][3];   /* parent translation */
    double mass[ORACLE_MAX_DOF];
    double com[ORACLE_MAX_DOF][3];
    double icom[ORACLE_MAX_DOF][9]; /* inertia about COM, row-major */
    double io[ORACLE_MAX_DOF][9];   /* inertia about link origin, row-major */
    /* 0: the reference's semantics -- joint poses rotate about `axis` but the motion
     *    subspace is hard-coded to z (multibody.rs:130-138, spatial.rs:180-185).
     * 1: general revolute axes (beyond the reference): S_i = (axis_i, 0)
     *    in RNEA / CRBA / jac.  Identical to 0 when every axis is +z.  Parity for non-z
     *    axes is pinned by the independent 6x6 formulation (featherstone6.py), not the
     *    reference (which has no consistent general-axis dynamics). */
    int general_axes;
    /* Kinematic tree (beyond the reference's serial chain): parent
     * link index (-1 = the fixed base; parent[i] < i, so index order is a topological
     * order) and joint type (0 revolute, 1 prismatic along `axis`).  Every constructor
     * sets the reference's serial revolute chain (parent[i] = i - 1); the algorithms then
     * perform exactly the operations of the serial code path. */
    int parent[ORACLE_MAX_DOF];
    int prismatic[ORACLE_MAX_DOF];
} oracle_model;

/* Raw per-revolute-joint URDF values, 16 doubles per joint:
 *   xyz[3] rpy[3] axis[3] mass com[3] ... then inertia6 (ixx ixy ixz iyy iyz izz) separately.
 * Follows RevoluteJoint::from_xurdf_joint (joint.rs:53-68). Returns 0 on success. */
int oracle_model_from_raw(oracle_model *m, int n,
                          const double *xyz, const double *rpy, const double *axis,
                          const double *mass, const double *com, const double *inertia6);

/* A chain given by explicit parent frames (R_p row-major 9 per link, p 3), unit-normalised
 * axes, and bodies (mass, com, inertia about the COM row-major 9) -- the form the merged
 * physical-tree URDF reading produces (oracle/urdf_model.py tree mode).  Returns 0. */
int oracle_model_from_frames(oracle_model *m, int n, const double *Rp, const double *p,
                             const double *axis, const double *mass, const double *com,
                             const double *icom9);
void oracle_model_set_general_axes(oracle_model *m, int on);
/* Tree topology and joint types (parent[i] in [-1, i), prismatic[i] in {0, 1}); NULL keeps
 * the current array.  Returns 0, or -1 on a bad parent / type. */
int oracle_model_set_topology(oracle_model *m, const int *parent, const int *prismatic);

int oracle_model_dof(const oracle_model *m);
int oracle_model_size(void);

/* Single-configuration algorithms (reference: multibody.rs). */
void oracle_rnea(const oracle_model *m, const double *q, const double *qd,
                 const double *qdd, double *tau);                       /* 111-153 */
void oracle_crba(const oracle_model *m, const double *q, double *H);    /* 155-174 */
void oracle_fwd_kin(const oracle_model *m, const double *q, double *pos); /* 87-93 */
void oracle_jac(const oracle_model *m, const double *q, double *J);     /* 95-108 */
/* qdd = sym(H)^-1 (tau - rnea(q,qd,0)); returns 0, or -1 if H is not SPD. */
int oracle_fd(const oracle_model *m, const double *q, const double *qd,
              const double *tau, double *qdd);

/* Fused rollout: K steps of semi-implicit Euler on the forward
 * dynamics definition: qd += dt * fd(q, qd, tau_k); q += dt * qd.  tau_seq is K x n
 * (step-major); q, qd are updated in place; traj (K x n, may be NULL) receives q after
 * each step.  Returns 0, or -1 if an H is not SPD. */
int oracle_rollout(const oracle_model *m, double *q, double *qd, const double *tau_seq,
                   double dt, int K, double *traj);
/* SoA batched rollout: q/qd [n][ld], tau_seq [K][n][ld], traj [K][n][ld] or NULL. */
void oracle_rollout_batch(const oracle_model *m, double *q, double *qd, const double *tau_seq,
                          double dt, int K, double *traj, long batch, long ld, int nthreads);

/* Batched SoA drivers (x[j*ld + b]) over `nthreads` OpenMP threads (<=0: all). */
void oracle_rnea_batch(const oracle_model *m, const double *q, const double *qd,
                       const double *qdd, double *tau, long batch, long ld, int nthreads);
void oracle_fd_batch(const oracle_model *m, const double *q, const double *qd,
                     const double *tau, double *qdd, long batch, long ld, int nthreads);
void oracle_crba_batch(const oracle_model *m, const double *q, double *H,
                       long batch, long ld, int nthreads);

/* Primitives exposed for the restated reference unit tests (spatial.rs:283-382). */
void oracle_quat_from_scaled_axis(const double v[3], double out_q[4]);
void oracle_quat_from_axis_angle(const double axis[3], double angle, double out_q[4]);
void oracle_quat_to_matrix(const double q[4], double R[9]);
void oracle_rotation_from_euler(double r, double p, double y, double R[9]);
void oracle_rotation_scaled_axis(const double R[9], double out[3]);
/* iso = {q[4], t[3]} packed as 7 doubles */
void oracle_motion_transform(const double iso[7], const double lin[3], const double rot[3],
                             double out_lin[3], double out_rot[3]);   /* spatial.rs:110-116 */
void oracle_force_transform(const double iso[7], const double lin[3], const double rot[3],
                            double out_lin[3], double out_rot[3]);    /* spatial.rs:242-248 */
void oracle_iso_inverse(const double iso[7], double out[7]);
void oracle_quat_rotate(const double q[4], const double v[3], double out[3]);

/* Count of quaternion/vector flops is not tracked; this returns the link-frame
 * parent transform (parent_to_child, joint.rs:36-38) as iso7. */
void oracle_parent_to_child(const oracle_model *m, int i, double qi, double iso_out[7]);

#ifdef __cplusplus
}
#endif
#endif
