// artinertia.hip.hpp -- 6x6 spatial / articulated inertia in 3x3 block form (device).
// Shared by aba.hip (articulated inertia) and crba.hip (composite inertia).
#pragma once

#include "spatial.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------ articulated-body (ABA) helpers
// Articulated inertia in block form [[A, B], [B^T, M]] acting on (rot, lin).
template <typename T>
struct ArtI {
    S3<T> A;
    M3<T> B;
    S3<T> M;
};

template <typename T>
RB_HD ArtI<T> rigid_inertia(const Link<T> &L) {
    // I_o, [h]x, m*1  (Inertia::to_matrix6 form, inertia.rs:53-70)
    ArtI<T> I;
    I.A = L.Io;
    I.B = M3<T>{{T(0), -L.h.z, L.h.y, L.h.z, T(0), -L.h.x, -L.h.y, L.h.x, T(0)}};
    I.M = S3<T>{L.m, T(0), T(0), L.m, T(0), L.m};
    return I;
}

// E S E^T for symmetric S
template <typename T>
RB_HD S3<T> rot_sym(const M3<T> &E, const S3<T> &S) {
    const T s[9] = {S.xx, S.xy, S.xz, S.xy, S.yy, S.yz, S.xz, S.yz, S.zz};
    T t[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            t[3 * r + c] = fmadd(E.m[3 * r + 0], s[c], fmadd(E.m[3 * r + 1], s[3 + c], E.m[3 * r + 2] * s[6 + c]));
    auto e = [&](int r, int c) {
        return fmadd(t[3 * r + 0], E.m[3 * c + 0], fmadd(t[3 * r + 1], E.m[3 * c + 1], t[3 * r + 2] * E.m[3 * c + 2]));
    };
    return S3<T>{e(0, 0), e(0, 1), e(0, 2), e(1, 1), e(1, 2), e(2, 2)};
}

// E B E^T for general B
template <typename T>
RB_HD M3<T> rot_full(const M3<T> &E, const M3<T> &Bm) {
    T t[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            t[3 * r + c] = fmadd(E.m[3 * r + 0], Bm.m[c], fmadd(E.m[3 * r + 1], Bm.m[3 + c], E.m[3 * r + 2] * Bm.m[6 + c]));
    M3<T> o;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            o.m[3 * r + c] = fmadd(t[3 * r + 0], E.m[3 * c + 0], fmadd(t[3 * r + 1], E.m[3 * c + 1], t[3 * r + 2] * E.m[3 * c + 2]));
    return o;
}

// X^T Ia X for the child->parent transform (E, p): rotate blocks, then shift by
// P = [p]x:  B'' = B' + P M',  A'' = A' + P B'^T + B'' P^T,  M'' = M'.
template <typename T>
RB_HD ArtI<T> to_parent(const M3<T> &E, const V3<T> &p, const ArtI<T> &I) {
    const S3<T> A1 = rot_sym(E, I.A);
    const M3<T> B1 = rot_full(E, I.B);
    const S3<T> M1 = rot_sym(E, I.M);
    const T m[9] = {M1.xx, M1.xy, M1.xz, M1.xy, M1.yy, M1.yz, M1.xz, M1.yz, M1.zz};
    M3<T> B2;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        // rows of P = [[0,-pz,py],[pz,0,-px],[-py,px,0]]
        B2.m[0 + c] = fmadd(-p.z, m[3 + c], fmadd(p.y, m[6 + c], B1.m[0 + c]));
        B2.m[3 + c] = fmadd(p.z, m[0 + c], fmadd(-p.x, m[6 + c], B1.m[3 + c]));
        B2.m[6 + c] = fmadd(-p.y, m[0 + c], fmadd(p.x, m[3 + c], B1.m[6 + c]));
    }
    const T P[9] = {T(0), -p.z, p.y, p.z, T(0), -p.x, -p.y, p.x, T(0)};
    // (P B1^T)[r][c] = sum_k P[r][k] B1[c][k];  (B2 P^T)[r][c] = sum_k B2[r][k] P[c][k]
    auto a = [&](int r, int c, T base) {
        T s = base;
#pragma unroll
        for (int k = 0; k < 3; ++k) s = fmadd(P[3 * r + k], B1.m[3 * c + k], s);
#pragma unroll
        for (int k = 0; k < 3; ++k) s = fmadd(B2.m[3 * r + k], P[3 * c + k], s);
        return s;
    };
    ArtI<T> o;
    o.A = S3<T>{a(0, 0, A1.xx), a(0, 1, A1.xy), a(0, 2, A1.xz), a(1, 1, A1.yy), a(1, 2, A1.yz), a(2, 2, A1.zz)};
    o.B = B2;
    o.M = M1;
    return o;
}

// Model-specialised kernels (RB_SPLIT_ROT, set by jit.cpp): E = R_p Rz(q) with R_p a
// compile-time constant, so E S E^T = R_p (Rz S Rz^T) R_p^T.  The Rz congruence of a
// symmetric S uses the double angle (C = cos 2q, S2 = sin 2q):
//   xx' = h + g C - xy S2,  yy' = h - g C + xy S2,  xy' = g S2 + xy C   (h, g = (xx +- yy)/2)
//   xz' = c xz - s yz,      yz' = s xz + c yz,      zz' = zz
// -- 10-14 FMAs where the folded E S E^T costs ~24 -- and the constant R_p congruence folds
// to relabelling / sign changes for the signed-permutation frames URDF joints usually have.
#ifndef RB_SPLIT_ROT
#define RB_SPLIT_ROT 0
#endif
template <typename T>
RB_HD S3<T> rot_sym_z(T c, T s, T C, T S2, const S3<T> &S) {
    const T h = T(0.5) * (S.xx + S.yy), g = T(0.5) * (S.xx - S.yy);
    return S3<T>{fmadd(g, C, fmadd(-S.xy, S2, h)), fmadd(g, S2, S.xy * C), fmadd(c, S.xz, -s * S.yz),
                 fmadd(-g, C, fmadd(S.xy, S2, h)), fmadd(s, S.xz, c * S.yz), S.zz};
}

// to_parent with the symmetric blocks rotated as R_p (Rz S Rz^T) R_p^T.
template <typename T>
RB_HD ArtI<T> to_parent_split(const M3<T> &Rp, T c, T s, const M3<T> &E, const V3<T> &p,
                                                   const ArtI<T> &I) {
    const T C = fmadd(c, c, -s * s), S2 = (c + c) * s;
    ArtI<T> J = I;
    J.A = rot_sym(Rp, rot_sym_z(c, s, C, S2, I.A));
    J.M = rot_sym(Rp, rot_sym_z(c, s, C, S2, I.M));
    // B and the shift as to_parent, with the rotated symmetric blocks passed through unchanged
    const M3<T> B1 = rot_full(E, I.B);
    const S3<T> M1 = J.M;
    const T m[9] = {M1.xx, M1.xy, M1.xz, M1.xy, M1.yy, M1.yz, M1.xz, M1.yz, M1.zz};
    M3<T> B2;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        B2.m[0 + k] = fmadd(-p.z, m[3 + k], fmadd(p.y, m[6 + k], B1.m[0 + k]));
        B2.m[3 + k] = fmadd(p.z, m[0 + k], fmadd(-p.x, m[6 + k], B1.m[3 + k]));
        B2.m[6 + k] = fmadd(-p.y, m[0 + k], fmadd(p.x, m[3 + k], B1.m[6 + k]));
    }
    const T P[9] = {T(0), -p.z, p.y, p.z, T(0), -p.x, -p.y, p.x, T(0)};
    auto a = [&](int r, int cc, T base) {
        T acc = base;
#pragma unroll
        for (int k = 0; k < 3; ++k) acc = fmadd(P[3 * r + k], B1.m[3 * cc + k], acc);
#pragma unroll
        for (int k = 0; k < 3; ++k) acc = fmadd(B2.m[3 * r + k], P[3 * cc + k], acc);
        return acc;
    };
    const S3<T> A1 = J.A;
    ArtI<T> o;
    o.A = S3<T>{a(0, 0, A1.xx), a(0, 1, A1.xy), a(0, 2, A1.xz), a(1, 1, A1.yy), a(1, 2, A1.yz), a(2, 2, A1.zz)};
    o.B = B2;
    o.M = M1;
    return o;
}

// ------------------------------------------------- composite rigid body (CRBA) helpers
// A composite of rigid bodies is rigid: mass m, first moment h = m c and the inertia I_o
// about the link origin (Inertia {mass, com, inertia}, inertia.rs:12-18) -- 10 values where
// the articulated block form carries 21, and m is a compile-time constant in the
// model-specialised kernels (a sum of link masses).
template <typename T>
struct RigidI {
    T m;
    V3<T> h;
    S3<T> Io;
};

template <typename T>
RB_HD RigidI<T> rigid_of(const Link<T> &L) {
    return RigidI<T>{L.m, L.h, L.Io};
}

// X^T I X for the child->parent transform (E, p) (Inertia::transform, inertia.rs:81-89):
// rotate, h1 = E h, Io1 = E Io E^T, then move the reference point by p (parallel axis):
//   h'  = h1 + m p
//   Io' = Io1 - (h1 p^T + p h1^T) - m p p^T + (2 p.h1 + m |p|^2) 1
// With RB_SPLIT_ROT the rotation is R_p (Rz S Rz^T) R_p^T (rot_sym_z), as to_parent_split.
template <typename T>
RB_HD RigidI<T> rigid_to_parent(const M3<T> &Rp, T c, T s, const M3<T> &E, const V3<T> &p, const RigidI<T> &I) {
    S3<T> Io1;
    V3<T> h1;
    if constexpr (RB_SPLIT_ROT != 0) {
        const T C = fmadd(c, c, -s * s), S2 = (c + c) * s;
        Io1 = rot_sym(Rp, rot_sym_z(c, s, C, S2, I.Io));
        h1 = mul(Rp, v3(fmadd(c, I.h.x, -s * I.h.y), fmadd(s, I.h.x, c * I.h.y), I.h.z));
    } else {
        Io1 = rot_sym(E, I.Io);
        h1 = mul(E, I.h);
    }
    const T m = I.m;
    const T d = fmadd(T(2) * p.x, h1.x, fmadd(T(2) * p.y, h1.y, fmadd(T(2) * p.z, h1.z,
                      m * fmadd(p.x, p.x, fmadd(p.y, p.y, p.z * p.z)))));
    const T mpx = m * p.x, mpy = m * p.y, mpz = m * p.z;
    RigidI<T> o;
    o.m = m;
    o.h = v3(h1.x + mpx, h1.y + mpy, h1.z + mpz);
    o.Io = S3<T>{fmadd(-(h1.x + h1.x + mpx), p.x, Io1.xx + d),
                 fmadd(-(h1.x + mpx), p.y, fmadd(-h1.y, p.x, Io1.xy)),
                 fmadd(-(h1.x + mpx), p.z, fmadd(-h1.z, p.x, Io1.xz)),
                 fmadd(-(h1.y + h1.y + mpy), p.y, Io1.yy + d),
                 fmadd(-(h1.y + mpy), p.z, fmadd(-h1.z, p.y, Io1.yz)),
                 fmadd(-(h1.z + h1.z + mpz), p.z, Io1.zz + d)};
    return o;
}

// The composite step of crba_core in one pass: X^T I X (inertia.rs:81-89) plus the parent
// link's own body (inertia.rs:96-105), for model-specialised kernels whose R_p is a constant
// signed permutation (RB_SPLIT_ROT) and whose constants fold (not RB_OPAQUE_CONSTS).  With
// P(h) = 2 (p.h) 1 - (h p^T + p h^T) (linear in h) and b = m p + h_parent:
//   h'  = R_p (Rz h + R_p^T b)
//   Io' = R_p (Rz Io Rz^T + K') R_p^T + P(h'),   K' = R_p^T (m (|p|^2 1 - p p^T) + Io_parent - P(b)) R_p
// so every constant is the innermost addend of an FMA chain instead of a separate add (the
// parent's 9 values, the parallel-axis constants).  The Rz congruence uses half the double
// angle, C = cos(2q)/2 = 1/2 - s^2 and S = sin(2q)/2 = c s, and the trace it keeps:
//   xx' = (xx + yy)/2 + w,  yy' = (xx + yy)/2 - w,  w = (xx - yy) C - 2 xy S
//   xy' = (xx - yy) S + 2 xy C,  xz' = c xz - s yz,  yz' = s xz + c yz,  zz' = zz.
// FR3 fp64: 27 instead of 33-35 VALU per composite step (tools/fd_stages.py).
template <typename T>
RB_HD M3<T> transpose(const M3<T> &R) {
    return M3<T>{{R.m[0], R.m[3], R.m[6], R.m[1], R.m[4], R.m[7], R.m[2], R.m[5], R.m[8]}};
}

template <typename T>
RB_HD S3<T> parallel_axis_p(const V3<T> &p, const V3<T> &h) {  // P(h) above
    return S3<T>{T(2) * fmadd(p.y, h.y, p.z * h.z), -fmadd(h.x, p.y, p.x * h.y), -fmadd(h.x, p.z, p.x * h.z),
                 T(2) * fmadd(p.x, h.x, p.z * h.z), -fmadd(h.y, p.z, p.y * h.z), T(2) * fmadd(p.x, h.x, p.y * h.y)};
}

// A folded model constant that enters as an FMA addend: pinned in SGPRs so the FMA reads it
// there (VOP3 src2).  Left to the compiler, a 64-bit addend is copied into a VGPR pair with two
// v_mov per use to feed the two-address v_fmac form (FR3 fp64: 55 extra VALU per launch).
template <typename T>
RB_HD T sconst(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_constant_p(v)) asm volatile("" : "+s"(v));
#endif
    return v;
}
RB_HD f2 sconst(f2 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_constant_p(v.x) && __builtin_constant_p(v.y) && v.x == v.y) {
        float c = v.x;
        asm volatile("" : "+s"(c));
        return f2{c, c};
    }
#endif
    return v;
}

template <typename T>
RB_HD RigidI<T> rigid_to_parent_add(const M3<T> &Rp, T c, T s, const V3<T> &p, const RigidI<T> &I,
                                    const Link<T> &Lp) {
    const T m = I.m;
    // constants (folded at compile time)
    const V3<T> b = v3(fmadd(m, p.x, Lp.h.x), fmadd(m, p.y, Lp.h.y), fmadd(m, p.z, Lp.h.z));
    const S3<T> Pb = parallel_axis_p(p, b);
    const S3<T> K{fmadd(m, fmadd(p.y, p.y, p.z * p.z), Lp.Io.xx) - Pb.xx, fmadd(-m, p.x * p.y, Lp.Io.xy) - Pb.xy,
                  fmadd(-m, p.x * p.z, Lp.Io.xz) - Pb.xz, fmadd(m, fmadd(p.x, p.x, p.z * p.z), Lp.Io.yy) - Pb.yy,
                  fmadd(-m, p.y * p.z, Lp.Io.yz) - Pb.yz, fmadd(m, fmadd(p.x, p.x, p.y * p.y), Lp.Io.zz) - Pb.zz};
    const M3<T> Rt = transpose(Rp);
    const S3<T> Kf = rot_sym(Rt, K);
    const V3<T> bf = mul(Rt, b);
    const S3<T> Kr{sconst(Kf.xx), sconst(Kf.xy), sconst(Kf.xz), sconst(Kf.yy), sconst(Kf.yz), sconst(Kf.zz)};
    const V3<T> br = v3(sconst(bf.x), sconst(bf.y), sconst(bf.z));
    // per configuration
    const S3<T> &S = I.Io;
    const T sum = S.xx + S.yy, dif = S.xx - S.yy, xy2 = S.xy + S.xy;
    const T C = fmadd(-s, s, T(0.5)), S2 = c * s;
    const T w = fmadd(dif, C, -(xy2 * S2));
    const S3<T> R{fmadd(T(0.5), sum, Kr.xx) + w, fmadd(dif, S2, fmadd(xy2, C, Kr.xy)),
                  fmadd(c, S.xz, fmadd(-s, S.yz, Kr.xz)), fmadd(T(0.5), sum, Kr.yy) - w,
                  fmadd(s, S.xz, fmadd(c, S.yz, Kr.yz)), S.zz + Kr.zz};
    const V3<T> hr = v3(fmadd(c, I.h.x, fmadd(-s, I.h.y, br.x)), fmadd(s, I.h.x, fmadd(c, I.h.y, br.y)), I.h.z + br.z);
    RigidI<T> o;
    o.m = m + Lp.m;
    o.h = mul(Rp, hr);
    const S3<T> Io1 = rot_sym(Rp, R);
    const V3<T> &h = o.h;
    o.Io = S3<T>{fmadd(T(2) * p.y, h.y, fmadd(T(2) * p.z, h.z, Io1.xx)), fmadd(-p.y, h.x, fmadd(-p.x, h.y, Io1.xy)),
                 fmadd(-p.z, h.x, fmadd(-p.x, h.z, Io1.xz)), fmadd(T(2) * p.x, h.x, fmadd(T(2) * p.z, h.z, Io1.yy)),
                 fmadd(-p.z, h.y, fmadd(-p.y, h.z, Io1.yz)), fmadd(T(2) * p.x, h.x, fmadd(T(2) * p.y, h.y, Io1.zz))};
    return o;
}

template <typename T>
RB_HD void add_rigid(RigidI<T> &I, const Link<T> &L) {
    I.m += L.m;
    I.h = v3(I.h.x + L.h.x, I.h.y + L.h.y, I.h.z + L.h.z);
    I.Io.xx += L.Io.xx; I.Io.xy += L.Io.xy; I.Io.xz += L.Io.xz;
    I.Io.yy += L.Io.yy; I.Io.yz += L.Io.yz; I.Io.zz += L.Io.zz;
}

template <typename T>
RB_HD void add_rigid(ArtI<T> &I, const Link<T> &L) {
    I.A.xx += L.Io.xx; I.A.xy += L.Io.xy; I.A.xz += L.Io.xz;
    I.A.yy += L.Io.yy; I.A.yz += L.Io.yz; I.A.zz += L.Io.zz;
    I.B.m[1] -= L.h.z; I.B.m[2] += L.h.y;
    I.B.m[3] += L.h.z; I.B.m[5] -= L.h.x;
    I.B.m[6] -= L.h.y; I.B.m[7] += L.h.x;
    I.M.xx += L.m; I.M.yy += L.m; I.M.zz += L.m;
}

}  // namespace dev
}  // namespace rbamd
