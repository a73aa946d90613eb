/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h for the parity-pinning story).
 *
 * fp64 restatement of khaninger/rigidbody-rs @ 2025-02-24.  Every function follows
 * the reference's own formulation and operation order: unit quaternions for the
 * link rotations (nalgebra 0.33.2 Isometry3<f64>), vectors rotated by the
 * quaternion sandwich nalgebra uses, and the spatial-algebra operators of
 * rigidbody/src/spatial.rs and inertia.rs.  It is deliberately *not* optimised:
 * it is the checker and the CPU baseline ("port"), never the product.
 *
 * nalgebra semantics restated here (third-party, pinned Cargo.lock:205-218):
 *   UnitQuaternion::from_scaled_axis(v) = exp(v/2) with identity below |v/2|<=eps
 *   UnitQuaternion * Vector3            = v + w*t + u x t,  t = 2 u x v
 *   Quaternion product                  = Hamilton product, coords (i, j, k, w)
 *   Rotation3::from_euler_angles(r,p,y) = Rz(y) Ry(p) Rx(r)
 *   Rotation3::scaled_axis              = normalised skew part * acos((tr-1)/2)
 *   Isometry3 compose / inverse         = (R1R2, t1+R1 t2) / (R^-1, -(R^-1 t))
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { double lin[3], rot[3]; } sv6;          /* SpatialVelocity / SpatialForce */
typedef struct { double q[4]; double t[3]; } iso3;      /* Isometry3, q = (i,j,k,w) */
typedef struct { double mass, com[3], icom[9], io[9]; } inertia_t; /* inertia.rs:12-18 */

static const double GRAVITY = 9.81; /* multibody.rs:117-120 */

/* ---------------------------------------------------------------- vectors -- */
static void cross3(const double a[3], const double b[3], double o[3]) {
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}

/* nalgebra Matrix3 * Vector3 (column-wise accumulate) on a row-major 3x3 */
static void matvec3(const double M[9], const double v[3], double o[3]) {
    double r0 = M[0] * v[0], r1 = M[3] * v[0], r2 = M[6] * v[0];
    r0 += M[1] * v[1]; r1 += M[4] * v[1]; r2 += M[7] * v[1];
    r0 += M[2] * v[2]; r1 += M[5] * v[2]; r2 += M[8] * v[2];
    o[0] = r0; o[1] = r1; o[2] = r2;
}

static void matmul3(const double A[9], const double B[9], double C[9]) {
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = A[3 * i + 0] * B[0 + j];
            s += A[3 * i + 1] * B[3 + j];
            s += A[3 * i + 2] * B[6 + j];
            T[3 * i + j] = s;
        }
    memcpy(C, T, sizeof T);
}

static void transpose3(const double A[9], double T[9]) {
    double U[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) U[3 * j + i] = A[3 * i + j];
    memcpy(T, U, sizeof U);
}

/* nalgebra Vector3::cross_matrix */
static void cross_matrix(const double v[3], double M[9]) {
    M[0] = 0.0;   M[1] = -v[2]; M[2] = v[1];
    M[3] = v[2];  M[4] = 0.0;   M[5] = -v[0];
    M[6] = -v[1]; M[7] = v[0];  M[8] = 0.0;
}

/* ------------------------------------------------------------ quaternions -- */
static void qmul(const double a[4], const double b[4], double o[4]) {
    /* (i, j, k, w) coords; nalgebra Quaternion Mul */
    double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    double i = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    double j = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
    double k = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
    o[0] = i; o[1] = j; o[2] = k; o[3] = w;
}

static void qconj(const double a[4], double o[4]) {
    o[0] = -a[0]; o[1] = -a[1]; o[2] = -a[2]; o[3] = a[3];
}

void oracle_quat_rotate(const double q[4], const double v[3], double out[3]) {
    double t[3], c[3];
    cross3(q, v, t);
    t[0] *= 2.0; t[1] *= 2.0; t[2] *= 2.0;
    cross3(q, t, c);
    double o0 = t[0] * q[3] + c[0] + v[0];
    double o1 = t[1] * q[3] + c[1] + v[1];
    double o2 = t[2] * q[3] + c[2] + v[2];
    out[0] = o0; out[1] = o1; out[2] = o2;
}

void oracle_quat_from_scaled_axis(const double v[3], double out[4]) {
    double h[3] = {v[0] / 2.0, v[1] / 2.0, v[2] / 2.0};
    double nn = h[0] * h[0] + h[1] * h[1] + h[2] * h[2];
    if (nn <= DBL_EPSILON * DBL_EPSILON) {
        out[0] = out[1] = out[2] = 0.0; out[3] = 1.0;
        return;
    }
    double w_exp = 1.0; /* exp(0) */
    double n = sqrt(nn);
    double s = w_exp * sin(n) / n;
    out[0] = h[0] * s; out[1] = h[1] * s; out[2] = h[2] * s;
    out[3] = w_exp * cos(n);
}

void oracle_quat_from_axis_angle(const double axis[3], double angle, double out[4]) {
    /* UnitQuaternion::from_axis_angle: (axis * sin(a/2), cos(a/2)) */
    double s = sin(angle / 2.0), c = cos(angle / 2.0);
    out[0] = axis[0] * s; out[1] = axis[1] * s; out[2] = axis[2] * s; out[3] = c;
}

void oracle_quat_to_matrix(const double q[4], double R[9]) {
    double i = q[0], j = q[1], k = q[2], w = q[3];
    double ww = w * w, ii = i * i, jj = j * j, kk = k * k;
    double ij = i * j * 2.0, wk = w * k * 2.0, wj = w * j * 2.0;
    double ik = i * k * 2.0, jk = j * k * 2.0, wi = w * i * 2.0;
    R[0] = ww + ii - jj - kk; R[1] = ij - wk;           R[2] = wj + ik;
    R[3] = wk + ij;           R[4] = ww - ii + jj - kk; R[5] = jk - wi;
    R[6] = ik - wj;           R[7] = wi + jk;           R[8] = ww - ii - jj + kk;
}

void oracle_rotation_from_euler(double roll, double pitch, double yaw, double R[9]) {
    double sr = sin(roll), cr = cos(roll);
    double sp = sin(pitch), cp = cos(pitch);
    double sy = sin(yaw), cy = cos(yaw);
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

void oracle_rotation_scaled_axis(const double R[9], double out[3]) {
    double ax[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    double n = sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    if (!(n > DBL_EPSILON)) { /* Unit::try_new(axis, default_epsilon) -> None */
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    double c = (R[0] + R[4] + R[8] - 1.0) / 2.0;
    if (c > 1.0) c = 1.0;
    if (c < -1.0) c = -1.0;
    double angle = acos(c);
    out[0] = ax[0] / n * angle; out[1] = ax[1] / n * angle; out[2] = ax[2] / n * angle;
}

/* -------------------------------------------------------------- isometry -- */
static void iso_mul(const iso3 *a, const iso3 *b, iso3 *o) {
    double rt[3], q[4];
    oracle_quat_rotate(a->q, b->t, rt);
    qmul(a->q, b->q, q);
    o->t[0] = a->t[0] + rt[0]; o->t[1] = a->t[1] + rt[1]; o->t[2] = a->t[2] + rt[2];
    memcpy(o->q, q, sizeof q);
}

static void iso_inv(const iso3 *a, iso3 *o) {
    double qi[4], nt[3] = {-a->t[0], -a->t[1], -a->t[2]}, t[3];
    qconj(a->q, qi);
    oracle_quat_rotate(qi, nt, t);
    memcpy(o->q, qi, sizeof qi);
    memcpy(o->t, t, sizeof t);
}

static iso3 iso_from7(const double x[7]) {
    iso3 r;
    memcpy(r.q, x, 4 * sizeof(double));
    memcpy(r.t, x + 4, 3 * sizeof(double));
    return r;
}

void oracle_iso_inverse(const double iso[7], double out[7]) {
    iso3 a = iso_from7(iso), b;
    iso_inv(&a, &b);
    memcpy(out, b.q, 4 * sizeof(double));
    memcpy(out + 4, b.t, 3 * sizeof(double));
}

/* ------------------------------------------------------- spatial algebra -- */
/* SpatialVelocity::transform, spatial.rs:110-116 */
static sv6 motion_tf(const iso3 *tr, const sv6 *v) {
    double qi[4], pxw[3], d[3];
    sv6 o;
    qconj(tr->q, qi);
    cross3(tr->t, v->rot, pxw);
    d[0] = v->lin[0] - pxw[0]; d[1] = v->lin[1] - pxw[1]; d[2] = v->lin[2] - pxw[2];
    oracle_quat_rotate(qi, d, o.lin);
    oracle_quat_rotate(qi, v->rot, o.rot);
    return o;
}

/* SpatialForce::transform, spatial.rs:242-248 */
static sv6 force_tf(const iso3 *tr, const sv6 *f) {
    double qi[4], pxf[3], d[3];
    sv6 o;
    qconj(tr->q, qi);
    oracle_quat_rotate(qi, f->lin, o.lin);
    cross3(tr->t, f->lin, pxf);
    d[0] = f->rot[0] - pxf[0]; d[1] = f->rot[1] - pxf[1]; d[2] = f->rot[2] - pxf[2];
    oracle_quat_rotate(qi, d, o.rot);
    return o;
}

void oracle_motion_transform(const double iso[7], const double lin[3], const double rot[3],
                             double out_lin[3], double out_rot[3]) {
    iso3 tr = iso_from7(iso);
    sv6 v, o;
    memcpy(v.lin, lin, sizeof v.lin);
    memcpy(v.rot, rot, sizeof v.rot);
    o = motion_tf(&tr, &v);
    memcpy(out_lin, o.lin, sizeof o.lin);
    memcpy(out_rot, o.rot, sizeof o.rot);
}

void oracle_force_transform(const double iso[7], const double lin[3], const double rot[3],
                            double out_lin[3], double out_rot[3]) {
    iso3 tr = iso_from7(iso);
    sv6 v, o;
    memcpy(v.lin, lin, sizeof v.lin);
    memcpy(v.rot, rot, sizeof v.rot);
    o = force_tf(&tr, &v);
    memcpy(out_lin, o.lin, sizeof o.lin);
    memcpy(out_rot, o.rot, sizeof o.rot);
}

/* SpatialVelocity::cross_star, spatial.rs:129-134 */
static sv6 cross_star(const sv6 *v, const sv6 *f) {
    sv6 o;
    double a[3], b[3];
    cross3(v->rot, f->lin, o.lin);
    cross3(v->rot, f->rot, a);
    cross3(v->lin, f->lin, b);
    o.rot[0] = a[0] + b[0]; o.rot[1] = a[1] + b[1]; o.rot[2] = a[2] + b[2];
    return o;
}

/* &Inertia * &SpatialVelocity, inertia.rs:107-117 (Featherstone eq. 2.63) */
static sv6 inertia_mul(const inertia_t *I, const sv6 *a) {
    sv6 o;
    double cxr[3], cxl[3], Ir[3];
    cross3(I->com, a->rot, cxr);
    cross3(I->com, a->lin, cxl);
    matvec3(I->io, a->rot, Ir);
    for (int k = 0; k < 3; ++k) {
        o.lin[k] = I->mass * a->lin[k] - I->mass * cxr[k];
        o.rot[k] = Ir[k] + I->mass * cxl[k];
    }
    return o;
}

/* Inertia::from_com, inertia.rs:21-35 */
static inertia_t inertia_from_com(double mass, const double com[3], const double icom[9]) {
    inertia_t I;
    double C[9], mC[9], CT[9], P[9];
    cross_matrix(com, C);
    for (int k = 0; k < 9; ++k) mC[k] = mass * C[k];
    transpose3(C, CT);
    matmul3(mC, CT, P);
    I.mass = mass;
    memcpy(I.com, com, sizeof I.com);
    memcpy(I.icom, icom, sizeof I.icom);
    for (int k = 0; k < 9; ++k) I.io[k] = icom[k] + P[k];
    return I;
}

/* Inertia::from_origin, inertia.rs:37-51 */
static inertia_t inertia_from_origin(double mass, const double com[3], const double io[9]) {
    inertia_t I;
    double C[9], mC[9], CT[9], P[9];
    cross_matrix(com, C);
    for (int k = 0; k < 9; ++k) mC[k] = mass * C[k];
    transpose3(C, CT);
    matmul3(mC, CT, P);
    I.mass = mass;
    memcpy(I.com, com, sizeof I.com);
    memcpy(I.io, io, sizeof I.io);
    for (int k = 0; k < 9; ++k) I.icom[k] = io[k] - P[k];
    return I;
}

/* Inertia::transform, inertia.rs:81-89 */
static inertia_t inertia_transform(const inertia_t *I, const iso3 *tr) {
    double R[9], RT[9], tmp[9], ic[9], c[3];
    oracle_quat_to_matrix(tr->q, R);
    oracle_quat_rotate(tr->q, I->com, c);
    c[0] += tr->t[0]; c[1] += tr->t[1]; c[2] += tr->t[2];
    transpose3(R, RT);
    matmul3(R, I->icom, tmp);
    matmul3(tmp, RT, ic);
    return inertia_from_com(I->mass, c, ic);
}

/* impl Add for Inertia, inertia.rs:96-105 */
static inertia_t inertia_add(const inertia_t *a, const inertia_t *b) {
    double com[3], io[9];
    double ms = a->mass + b->mass;
    for (int k = 0; k < 3; ++k) com[k] = (a->mass * a->com[k] + b->mass * b->com[k]) / ms;
    for (int k = 0; k < 9; ++k) io[k] = a->io[k] + b->io[k];
    return inertia_from_origin(ms, com, io);
}

static inertia_t body_of(const oracle_model *m, int i) {
    inertia_t I;
    I.mass = m->mass[i];
    memcpy(I.com, m->com[i], sizeof I.com);
    memcpy(I.icom, m->icom[i], sizeof I.icom);
    memcpy(I.io, m->io[i], sizeof I.io);
    return I;
}

/* ----------------------------------------------------------------- model -- */
int oracle_model_size(void) { return (int)sizeof(oracle_model); }
int oracle_model_dof(const oracle_model *m) { return m->n; }

/* RevoluteJoint::from_xurdf_joint, joint.rs:53-68 */
int oracle_model_from_raw(oracle_model *m, int n,
                          const double *xyz, const double *rpy, const double *axis,
                          const double *mass, const double *com, const double *inertia6) {
    if (n < 1 || n > ORACLE_MAX_DOF) return -1;
    memset(m, 0, sizeof *m);
    m->n = n;
    for (int i = 0; i < n; ++i) {
        const double *a = axis + 3 * i;
        double an = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (!(an > 0.0)) return -2;
        for (int k = 0; k < 3; ++k) m->axis[i][k] = a[k] / an;
        double R[9], sa[3];
        oracle_rotation_from_euler(rpy[3 * i + 0], rpy[3 * i + 1], rpy[3 * i + 2], R);
        oracle_rotation_scaled_axis(R, sa);
        oracle_quat_from_scaled_axis(sa, m->pq[i]);
        memcpy(m->pt[i], xyz + 3 * i, 3 * sizeof(double));
        const double *J = inertia6 + 6 * i;
        double ic[9] = {J[0], J[1], J[2], J[1], J[3], J[4], J[2], J[4], J[5]};
        inertia_t I = inertia_from_com(mass[i], com + 3 * i, ic);
        m->mass[i] = I.mass;
        memcpy(m->com[i], I.com, sizeof I.com);
        memcpy(m->icom[i], I.icom, sizeof I.icom);
        memcpy(m->io[i], I.io, sizeof I.io);
        m->parent[i] = i - 1;
    }
    return 0;
}

/* Rotation matrix -> unit quaternion (i, j, k, w), Shepperd's branch on the largest
 * diagonal term; w >= 0. */
static void quat_from_matrix(const double R[9], double q[4]) {
    const double tr = R[0] + R[4] + R[8];
    double i, j, k, w;
    if (tr > 0.0) {
        double s = sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s; i = (R[7] - R[5]) / s; j = (R[2] - R[6]) / s; k = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        double s = sqrt(1.0 + R[0] - R[4] - R[8]) * 2.0;
        w = (R[7] - R[5]) / s; i = 0.25 * s; j = (R[1] + R[3]) / s; k = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        double s = sqrt(1.0 + R[4] - R[0] - R[8]) * 2.0;
        w = (R[2] - R[6]) / s; i = (R[1] + R[3]) / s; j = 0.25 * s; k = (R[5] + R[7]) / s;
    } else {
        double s = sqrt(1.0 + R[8] - R[0] - R[4]) * 2.0;
        w = (R[3] - R[1]) / s; i = (R[2] + R[6]) / s; j = (R[5] + R[7]) / s; k = 0.25 * s;
    }
    double nrm = sqrt(i * i + j * j + k * k + w * w);
    if (w < 0.0) nrm = -nrm;
    q[0] = i / nrm; q[1] = j / nrm; q[2] = k / nrm; q[3] = w / nrm;
}

int oracle_model_from_frames(oracle_model *m, int n, const double *Rp, const double *p,
                             const double *axis, const double *mass, const double *com,
                             const double *icom9) {
    if (n < 1 || n > ORACLE_MAX_DOF) return -1;
    memset(m, 0, sizeof *m);
    m->n = n;
    for (int i = 0; i < n; ++i) {
        const double *a = axis + 3 * i;
        double an = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (!(an > 0.0)) return -2;
        for (int k = 0; k < 3; ++k) m->axis[i][k] = a[k] / an;
        quat_from_matrix(Rp + 9 * i, m->pq[i]);
        memcpy(m->pt[i], p + 3 * i, 3 * sizeof(double));
        inertia_t I = inertia_from_com(mass[i], com + 3 * i, icom9 + 9 * i);
        m->mass[i] = I.mass;
        memcpy(m->com[i], I.com, sizeof I.com);
        memcpy(m->icom[i], I.icom, sizeof I.icom);
        memcpy(m->io[i], I.io, sizeof I.io);
        m->parent[i] = i - 1;
    }
    return 0;
}

void oracle_model_set_general_axes(oracle_model *m, int on) { m->general_axes = on != 0; }

int oracle_model_set_topology(oracle_model *m, const int *parent, const int *prismatic) {
    for (int i = 0; i < m->n; ++i) {
        if (parent && (parent[i] < -1 || parent[i] >= i)) return -1;
        if (prismatic && prismatic[i] != 0 && prismatic[i] != 1) return -1;
    }
    for (int i = 0; i < m->n; ++i) {
        if (parent) m->parent[i] = parent[i];
        if (prismatic) m->prismatic[i] = prismatic[i];
    }
    return 0;
}

/* Motion subspace of joint i: the reference's z (spatial.rs:180-185) or the true axis. */
static void joint_axis(const oracle_model *m, int i, double s[3]) {
    if (m->general_axes) {
        s[0] = m->axis[i][0]; s[1] = m->axis[i][1]; s[2] = m->axis[i][2];
    } else {
        s[0] = 0.0; s[1] = 0.0; s[2] = 1.0;
    }
}

/* RevoluteJoint::parent_to_child, joint.rs:36-38, 48-50 */
static iso3 parent_to_child(const oracle_model *m, int i, double qi) {
    iso3 r;
    double sa[3] = {m->axis[i][0] * qi, m->axis[i][1] * qi, m->axis[i][2] * qi};
    double jq[4];
    if (m->prismatic[i]) {
        /* prismatic: the joint origin, then a translation by axis * q in the joint frame */
        double d[3];
        oracle_quat_rotate(m->pq[i], sa, d);
        memcpy(r.q, m->pq[i], sizeof r.q);
        for (int k = 0; k < 3; ++k) r.t[k] = m->pt[i][k] + d[k];
        return r;
    }
    oracle_quat_from_scaled_axis(sa, jq);
    qmul(m->pq[i], jq, r.q);
    memcpy(r.t, m->pt[i], sizeof r.t);
    return r;
}

void oracle_parent_to_child(const oracle_model *m, int i, double qi, double iso_out[7]) {
    iso3 r = parent_to_child(m, i, qi);
    memcpy(iso_out, r.q, 4 * sizeof(double));
    memcpy(iso_out + 4, r.t, 3 * sizeof(double));
}

/* MBTransforms::from_joint_angles, multibody.rs:41-49 */
static void get_transforms(const oracle_model *m, const double *q, iso3 *tr) {
    for (int i = 0; i < m->n; ++i) tr[i] = parent_to_child(m, i, q[i]);
}

/* ------------------------------------------------------------ algorithms -- */
/* Multibody::rnea, multibody.rs:111-153 */
static void rnea_tr(const oracle_model *m, const iso3 *tr, const double *dq,
                    const double *ddq, double *tau) {
    sv6 f[ORACLE_MAX_DOF], V[ORACLE_MAX_DOF], A[ORACLE_MAX_DOF];
    const sv6 v0 = {{0, 0, 0}, {0, 0, 0}};
    const sv6 a0 = {{0, 0, GRAVITY}, {0, 0, 0}};
    for (int i = 0; i < m->n; ++i) {
        const int p = m->parent[i]; /* serial chain: i - 1 */
        sv6 v = motion_tf(&tr[i], p < 0 ? &v0 : &V[p]);
        sv6 a = motion_tf(&tr[i], p < 0 ? &a0 : &A[p]);
        if (m->prismatic[i]) {
            /* v += S qd; a += S qdd + v x (S qd), S = (rot 0, lin s) */
            double s[3], c[3];
            joint_axis(m, i, s);
            for (int k = 0; k < 3; ++k) v.lin[k] += s[k] * dq[i];
            for (int k = 0; k < 3; ++k) a.lin[k] += s[k] * ddq[i];
            cross3(v.rot, s, c);
            for (int k = 0; k < 3; ++k) a.lin[k] += c[k] * dq[i];
        } else if (!m->general_axes) {
            /* multibody.rs:126-138, z hard-coded */
            v.rot[2] += dq[i];
            a.rot[2] += ddq[i];
            a.lin[0] += v.lin[1] * dq[i];
            a.lin[1] += -v.lin[0] * dq[i];
            a.rot[0] += v.rot[1] * dq[i];
            a.rot[1] += -v.rot[0] * dq[i];
        } else {
            /* v += S qd; a += S qdd + v x (S qd), S = (rot s, lin 0) */
            double s[3], c[3];
            joint_axis(m, i, s);
            for (int k = 0; k < 3; ++k) v.rot[k] += s[k] * dq[i];
            for (int k = 0; k < 3; ++k) a.rot[k] += s[k] * ddq[i];
            cross3(v.lin, s, c);
            for (int k = 0; k < 3; ++k) a.lin[k] += c[k] * dq[i];
            cross3(v.rot, s, c);
            for (int k = 0; k < 3; ++k) a.rot[k] += c[k] * dq[i];
        }
        V[i] = v;
        A[i] = a;
        inertia_t I = body_of(m, i);
        sv6 Ia = inertia_mul(&I, &a);
        sv6 Iv = inertia_mul(&I, &v);
        sv6 cs = cross_star(&v, &Iv);
        for (int k = 0; k < 3; ++k) {
            f[i].lin[k] = Ia.lin[k] + cs.lin[k];
            f[i].rot[k] = Ia.rot[k] + cs.rot[k];
        }
    }
    for (int i = m->n - 1; i >= 0; --i) {
        double s[3];
        joint_axis(m, i, s);
        if (m->prismatic[i])
            tau[i] = s[0] * f[i].lin[0] + s[1] * f[i].lin[1] + s[2] * f[i].lin[2];
        else
            tau[i] = m->general_axes ? s[0] * f[i].rot[0] + s[1] * f[i].rot[1] + s[2] * f[i].rot[2] : f[i].rot[2];
        const int p = m->parent[i];
        if (p >= 0) {
            iso3 inv;
            iso_inv(&tr[i], &inv);
            sv6 ft = force_tf(&inv, &f[i]);
            for (int k = 0; k < 3; ++k) {
                f[p].lin[k] += ft.lin[k];
                f[p].rot[k] += ft.rot[k];
            }
        }
    }
}

void oracle_rnea(const oracle_model *m, const double *q, const double *qd,
                 const double *qdd, double *tau) {
    iso3 tr[ORACLE_MAX_DOF];
    get_transforms(m, q, tr);
    rnea_tr(m, tr, qd, qdd, tau);
}

/* Multibody::crba, multibody.rs:155-174.  H is n x n column-major; identity init,
 * so the strictly-lower triangle stays exactly 0 (156, 166). */
void oracle_crba(const oracle_model *m, const double *q, double *H) {
    int n = m->n;
    iso3 tr[ORACLE_MAX_DOF];
    get_transforms(m, q, tr);
    for (int c = 0; c < n; ++c)
        for (int r = 0; r < n; ++r) H[r + n * c] = (r == c) ? 1.0 : 0.0;
    /* composite inertias; in a tree a parent's entry accumulates each child's (for the
     * serial chain this is exactly body(i-1) + moved, multibody.rs:170) */
    inertia_t Ic[ORACLE_MAX_DOF];
    for (int i = 0; i < n; ++i) Ic[i] = body_of(m, i);
    for (int i = n - 1; i >= 0; --i) {
        const inertia_t I = Ic[i];
        sv6 S = {{0, 0, 0}, {0, 0, 0}}; /* BodyJacobian::revolute_z, spatial.rs:180-185 */
        joint_axis(m, i, m->prismatic[i] ? S.lin : S.rot);
        if (m->prismatic[i]) {
            sv6 F0 = inertia_mul(&I, &S);
            H[i + n * i] = S.lin[0] * F0.lin[0] + S.lin[1] * F0.lin[1] + S.lin[2] * F0.lin[2];
        } else if (!m->general_axes) {
            H[i + n * i] = I.io[8]; /* get_rotz, inertia.rs:91-93 */
        } else {
            double Is[3];
            matvec3(I.io, S.rot, Is);
            H[i + n * i] = S.rot[0] * Is[0] + S.rot[1] * Is[1] + S.rot[2] * Is[2];
        }
        sv6 F = inertia_mul(&I, &S);
        /* carry F to every ancestor j of i (serial: j = i-1 .. 0, multibody.rs:163-168) */
        for (int c = i, j = m->parent[i]; j >= 0; c = j, j = m->parent[j]) {
            iso3 inv;
            iso_inv(&tr[c], &inv);
            F = force_tf(&inv, &F);
            double sj[3];
            joint_axis(m, j, sj);
            if (m->prismatic[j])
                H[j + n * i] = sj[0] * F.lin[0] + sj[1] * F.lin[1] + sj[2] * F.lin[2];
            else
                H[j + n * i] = m->general_axes ? sj[0] * F.rot[0] + sj[1] * F.rot[1] + sj[2] * F.rot[2] : F.rot[2];
        }
        const int p = m->parent[i];
        if (p >= 0) {
            inertia_t moved = inertia_transform(&I, &tr[i]);
            inertia_t parent = Ic[p];
            Ic[p] = inertia_add(&parent, &moved);
        }
    }
}

/* Multibody::fwd_kin, multibody.rs:87-93 (ABI returns translation only, lib.rs:54-55) */
void oracle_fwd_kin(const oracle_model *m, const double *q, double *pos) {
    iso3 tr[ORACLE_MAX_DOF];
    get_transforms(m, q, tr);
    iso3 acc = {{0, 0, 0, 1}, {0, 0, 0}};
    /* the last link's ancestors, leaf to root (serial: n-1 .. 0) */
    for (int i = m->n - 1; i >= 0; i = m->parent[i]) {
        iso3 nxt;
        iso_mul(&tr[i], &acc, &nxt);
        acc = nxt;
    }
    memcpy(pos, acc.t, 3 * sizeof(double));
}

/* Multibody::jac, multibody.rs:95-108: 6 x n column-major, rows [lin; rot] */
void oracle_jac(const oracle_model *m, const double *q, double *J) {
    iso3 tr[ORACLE_MAX_DOF];
    get_transforms(m, q, tr);
    iso3 acc = {{0, 0, 0, 1}, {0, 0, 0}};
    memset(J, 0, 6 * (size_t)m->n * sizeof(double)); /* joints off the last link's path */
    for (int i = m->n - 1; i >= 0; i = m->parent[i]) {
        sv6 S = {{0, 0, 0}, {0, 0, 0}};
        joint_axis(m, i, m->prismatic[i] ? S.lin : S.rot);
        sv6 v = motion_tf(&acc, &S);
        for (int k = 0; k < 3; ++k) {
            J[6 * i + k] = v.lin[k];
            J[6 * i + 3 + k] = v.rot[k];
        }
        iso3 nxt;
        iso_mul(&tr[i], &acc, &nxt);
        acc = nxt;
    }
}

/* Forward dynamics definition: qdd = sym(H)^-1 (tau - rnea(q,qd,0)).
 * Cholesky on the symmetrised CRBA matrix. */
int oracle_fd(const oracle_model *m, const double *q, const double *qd,
              const double *tau, double *qdd) {
    int n = m->n;
    double H[ORACLE_MAX_DOF * ORACLE_MAX_DOF], L[ORACLE_MAX_DOF * ORACLE_MAX_DOF];
    double zero[ORACLE_MAX_DOF], b[ORACLE_MAX_DOF], y[ORACLE_MAX_DOF];
    memset(zero, 0, sizeof zero);
    oracle_crba(m, q, H);
    oracle_rnea(m, q, qd, zero, b);
    for (int i = 0; i < n; ++i) b[i] = tau[i] - b[i];
    /* symmetric A[r][c] from the upper triangle (col-major H) */
    for (int c = 0; c < n; ++c)
        for (int r = 0; r < n; ++r) {
            double v = (r <= c) ? H[r + n * c] : H[c + n * r];
            L[r * n + c] = v; /* row-major working copy */
        }
    for (int j = 0; j < n; ++j) {
        double d = L[j * n + j];
        for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
        if (!(d > 0.0)) return -1;
        d = sqrt(d);
        L[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = L[i * n + j];
            for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = s / d;
        }
    }
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * y[k];
        y[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * qdd[k];
        qdd[i] = s / L[i * n + i];
    }
    return 0;
}

/* Fused rollout: semi-implicit Euler on oracle_fd. */
int oracle_rollout(const oracle_model *m, double *q, double *qd, const double *tau_seq,
                   double dt, int K, double *traj) {
    int n = m->n;
    double qdd[ORACLE_MAX_DOF];
    for (int k = 0; k < K; ++k) {
        if (oracle_fd(m, q, qd, tau_seq + (long)k * n, qdd) != 0) return -1;
        for (int j = 0; j < n; ++j) {
            qd[j] += dt * qdd[j];
            q[j] += dt * qd[j];
        }
        if (traj)
            for (int j = 0; j < n; ++j) traj[(long)k * n + j] = q[j];
    }
    return 0;
}

/* ---------------------------------------------------------- batch drivers -- */
static int pick_threads(int nthreads) {
#ifdef _OPENMP
    return nthreads > 0 ? nthreads : omp_get_max_threads();
#else
    (void)nthreads;
    return 1;
#endif
}

void oracle_rnea_batch(const oracle_model *m, const double *q, const double *qd,
                       const double *qdd, double *tau, long batch, long ld, int nthreads) {
    int n = m->n;
    int nt = pick_threads(nthreads);
    (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (long b = 0; b < batch; ++b) {
        double x[ORACLE_MAX_DOF], y[ORACLE_MAX_DOF], z[ORACLE_MAX_DOF], t[ORACLE_MAX_DOF];
        for (int j = 0; j < n; ++j) {
            x[j] = q[j * ld + b]; y[j] = qd[j * ld + b]; z[j] = qdd[j * ld + b];
        }
        oracle_rnea(m, x, y, z, t);
        for (int j = 0; j < n; ++j) tau[j * ld + b] = t[j];
    }
}

void oracle_fd_batch(const oracle_model *m, const double *q, const double *qd,
                     const double *tau, double *qdd, long batch, long ld, int nthreads) {
    int n = m->n;
    int nt = pick_threads(nthreads);
    (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (long b = 0; b < batch; ++b) {
        double x[ORACLE_MAX_DOF], y[ORACLE_MAX_DOF], z[ORACLE_MAX_DOF], t[ORACLE_MAX_DOF];
        for (int j = 0; j < n; ++j) {
            x[j] = q[j * ld + b]; y[j] = qd[j * ld + b]; z[j] = tau[j * ld + b];
        }
        if (oracle_fd(m, x, y, z, t) != 0)
            for (int j = 0; j < n; ++j) t[j] = NAN;
        for (int j = 0; j < n; ++j) qdd[j * ld + b] = t[j];
    }
}

void oracle_crba_batch(const oracle_model *m, const double *q, double *H,
                       long batch, long ld, int nthreads) {
    int n = m->n;
    int nt = pick_threads(nthreads);
    (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (long b = 0; b < batch; ++b) {
        double x[ORACLE_MAX_DOF], h[ORACLE_MAX_DOF * ORACLE_MAX_DOF];
        for (int j = 0; j < n; ++j) x[j] = q[j * ld + b];
        oracle_crba(m, x, h);
        for (int e = 0; e < n * n; ++e) H[e * ld + b] = h[e];
    }
}

void oracle_rollout_batch(const oracle_model *m, double *q, double *qd, const double *tau_seq,
                          double dt, int K, double *traj, long batch, long ld, int nthreads) {
    int n = m->n;
    int nt = pick_threads(nthreads);
    (void)nt;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (long b = 0; b < batch; ++b) {
        double x[ORACLE_MAX_DOF], y[ORACLE_MAX_DOF];
        double t[64 * ORACLE_MAX_DOF], tr[64 * ORACLE_MAX_DOF];
        for (int j = 0; j < n; ++j) { x[j] = q[j * ld + b]; y[j] = qd[j * ld + b]; }
        for (int k0 = 0; k0 < K; k0 += 64) {
            int kk = K - k0 < 64 ? K - k0 : 64;
            for (int k = 0; k < kk; ++k)
                for (int j = 0; j < n; ++j) t[k * n + j] = tau_seq[((long)(k0 + k) * n + j) * ld + b];
            if (oracle_rollout(m, x, y, t, dt, kk, tr) != 0)
                for (int j = 0; j < n; ++j) { x[j] = NAN; y[j] = NAN; }
            if (traj)
                for (int k = 0; k < kk; ++k)
                    for (int j = 0; j < n; ++j) traj[((long)(k0 + k) * n + j) * ld + b] = tr[k * n + j];
        }
        for (int j = 0; j < n; ++j) { q[j * ld + b] = x[j]; qd[j * ld + b] = y[j]; }
    }
}
