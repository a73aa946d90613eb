// tree_body.hip.hpp -- kinematic trees and prismatic joints (device).  SURVEY §8(f) rank 4,
// beyond the reference, whose Multibody is a serial chain of revolute joints
// (multibody.rs:32, 111-174).  The per-link algebra is the serial code's (spatial.hip.hpp);
// what changes is where a link's parent state comes from and which spatial axis the joint
// moves along:
//   RNEA  Featherstone Table 5.1 with lambda(i):  v_i = X_i v_lambda(i) + S_i qd_i ...,
//         f_lambda(i) += X_i^T f_i
//   ABA   Table 7.1: articulated inertias / bias forces accumulate into the parent
//   CRBA  Table 6.2: composite inertias accumulate into the parent; H_ij != 0 only for j an
//         ancestor of i (upper triangle, the ABI's layout; everything else exact zeros)
//   FK / body Jacobian of the last link: its ancestor path only (other columns zero)
//
// The topology is a compile-time policy `Topo` (jit.cpp emits it from the model): parent(j),
// prismatic(j), last_child(j) (the highest-index child, -1 for a leaf), on_path(j)
// (ancestor-or-self of link N-1), is_ancestor(a, i) and child_toward(a, i) (a's child on the
// path down to i).  Every loop below is a compile-time loop (cfor), so each
// parent index and joint type is a constant: a link's state stays in registers exactly as
// long as a later child reads it, and a prismatic joint costs no runtime branch.  The
// serial revolute chain keeps its own tuned code (rnea_body / aba_body / crba_body); these
// forms run only for models the precompiled kernels cannot express.
#pragma once

#include "artinertia.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------------- compile-time loops
template <int V>
struct IC {
    static constexpr int value = V;
};

template <int I, int N, typename F>
RB_HD void cfor(F &&f) {
    if constexpr (I < N) {
        f(IC<I>{});
        cfor<I + 1, N>(f);
    }
}

// f(I-1), f(I-2), ..., f(0)
template <int I, typename F>
RB_HD void cfor_rev(F &&f) {
    if constexpr (I > 0) {
        f(IC<I - 1>{});
        cfor_rev<I - 1>(f);
    }
}

// Link frame in its parent: E = R_p Rz(q) and r = p for a revolute joint; E = R_p and
// r = p + R_p e_z q for a prismatic one (the model packer has already turned every joint
// axis into local z, model.cpp pack).
template <typename T, bool PRISMATIC>
RB_HD void link_frame(const Link<T> &L, T q, T c, T s, M3<T> &E, V3<T> &r) {
    if constexpr (PRISMATIC) {
        E = L.Rp;
        r = v3(fmadd(L.Rp.m[2], q, L.p.x), fmadd(L.Rp.m[5], q, L.p.y), fmadd(L.Rp.m[8], q, L.p.z));
    } else {
        E = joint_rotation(L.Rp, c, s);
        r = L.p;
    }
}

template <typename T>
RB_HD V3<T> add3(const V3<T> &a, const V3<T> &b) {
    return v3(a.x + b.x, a.y + b.y, a.z + b.z);
}

template <typename T>
RB_HD void add_art(ArtI<T> &I, const ArtI<T> &J) {
    I.A = S3<T>{I.A.xx + J.A.xx, I.A.xy + J.A.xy, I.A.xz + J.A.xz, I.A.yy + J.A.yy, I.A.yz + J.A.yz, I.A.zz + J.A.zz};
#pragma unroll
    for (int k = 0; k < 9; ++k) I.B.m[k] += J.B.m[k];
    I.M = S3<T>{I.M.xx + J.M.xx, I.M.xy + J.M.xy, I.M.xz + J.M.xz, I.M.yy + J.M.yy, I.M.yz + J.M.yz, I.M.zz + J.M.zz};
}

// Child -> parent force transform (spatial.rs:242-248 with the isometry inverse):
// f' = E f,  n' = E n + r x f'
template <typename T>
RB_HD void force_to_parent(const M3<T> &E, const V3<T> &r, V3<T> &n, V3<T> &f) {
    const V3<T> fl = mul(E, f);
    n = cross_add(mul(E, n), r, fl);
    f = fl;
}

// ----------------------------------------------------------------------------- RNEA
template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void rnea_eval_tree(const T *mdl, const T (&qv)[N], const T (&qdv)[N],
                                               const T (&qddv)[N], Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<Topo>(qv);
    gd.vals(qdv);
    gd.vals(qddv);
    auto out = [&](int j, T v) { out_(j, gd.out(v)); };
    T cs[N], sn[N];
    V3<T> W[N], V[N], AW[N], AV[N];  // link velocity / acceleration (rot, lin), link coordinates
    V3<T> fn[N], ff[N];              // per-link spatial force (moment, force)
    cfor<0, N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int p = Topo::parent(j);
        constexpr bool pri = Topo::prismatic(j);
        const Link<T> L = load_link(mdl, j);
        if constexpr (!pri) sin_cos<FAST>(qv[j], sn[j], cs[j]); else { cs[j] = T(1); sn[j] = T(0); }
        M3<T> E;
        V3<T> r;
        link_frame<T, pri>(L, qv[j], cs[j], sn[j], E, r);
        const T qdj = qdv[j];
        V3<T> w, v, aw, av;
        if constexpr (p < 0) {  // base: v = 0, a = (0, (0,0,+g)) -- multibody.rs:116-120
            const T g = T(kGravity);
            w = v3(T(0), T(0), T(0));
            v = w;
            aw = w;
            av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);
        } else {  // SpatialVelocity::transform (spatial.rs:110-116) of the parent's v and a
            w = mul_t(E, W[p]);
            v = mul_t(E, cross_sub(V[p], r, W[p]));
            aw = mul_t(E, AW[p]);
            av = mul_t(E, cross_sub(AV[p], r, AW[p]));
        }
        if constexpr (!pri) {  // S = (e_z, 0): multibody.rs:130-138
            w.z += qdj;
            aw.z += qddv[j];
            av.x = fmadd(v.y, qdj, av.x);
            av.y = fmadd(-v.x, qdj, av.y);
            aw.x = fmadd(w.y, qdj, aw.x);
            aw.y = fmadd(-w.x, qdj, aw.y);
        } else {  // S = (0, e_z): v.lin += e_z qd, a.lin += e_z qdd + w x e_z qd
            v.z += qdj;
            av.z += qddv[j];
            av.x = fmadd(w.y, qdj, av.x);
            av.y = fmadd(-w.x, qdj, av.y);
        }
        W[j] = w;
        V[j] = v;
        AW[j] = aw;
        AV[j] = av;
        // f = I a + v x* (I v)   (multibody.rs:140)
        link_force(L, j, w, v, aw, av, fn[j], ff[j]);
    });
    reload_fence();
    cfor_rev<N>([&](auto jc) {  // tau_j = S_j^T f_j; f_parent += X_j^T f_j  (multibody.rs:143-150)
        constexpr int j = decltype(jc)::value;
        constexpr int p = Topo::parent(j);
        constexpr bool pri = Topo::prismatic(j);
        out(j, pri ? ff[j].z : fn[j].z);
        if constexpr (p >= 0) {
            const Link<T> L = load_link(mdl, j);
            M3<T> E;
            V3<T> r;
            link_frame<T, pri>(L, qv[j], cs[j], sn[j], E, r);
            V3<T> n = fn[j], f = ff[j];
            force_to_parent(E, r, n, f);
            fn[p] = add3(fn[p], n);
            ff[p] = add3(ff[p], f);
        }
    });
}

// ------------------------------------------------------------------------------ ABA
// Featherstone Table 7.1 over the tree, in the 3x3 block form of aba_body.hip.hpp.  U = I^A S
// is (A e_z; B^T e_z) for a revolute joint and (B e_z; M e_z) for a prismatic one; the
// projected inertia I^a = I^A - U U^T / D annihilates S, so the corresponding row/column
// is written as exact zeros (as the serial kernel does).
template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void aba_eval_tree(const T *mdl, const T (&qv)[N], const T (&qdv)[N], const T (&tv)[N],
                                              Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<Topo>(qv);
    gd.vals(qdv);
    gd.vals(tv);
    auto out = [&](int j, T v) { out_(j, gd.out(v)); };
    T cs[N], sn[N];
    V3<T> W[N], V[N];                  // pass-1 velocities (read by children)
    T cw0[N], cw1[N], cv0[N], cv1[N];  // c_i = v_i x (S qd_i), nonzero entries
    V3<T> pn[N], pf[N];                // bias forces p_i = v_i x* (I_i v_i)
    cfor<0, N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int p = Topo::parent(j);
        constexpr bool pri = Topo::prismatic(j);
        const Link<T> L = load_link(mdl, j);
        if constexpr (!pri) sin_cos<FAST>(qv[j], sn[j], cs[j]); else { cs[j] = T(1); sn[j] = T(0); }
        const T qdj = qdv[j];
        V3<T> w, v;
        if constexpr (p < 0) {
            w = v3(T(0), T(0), T(0));
            v = w;
        } else {
            M3<T> E;
            V3<T> r;
            link_frame<T, pri>(L, qv[j], cs[j], sn[j], E, r);
            w = mul_t(E, W[p]);
            v = mul_t(E, cross_sub(V[p], r, W[p]));
        }
        if constexpr (!pri) {
            w.z += qdj;
            cw0[j] = w.y * qdj; cw1[j] = -w.x * qdj;
            cv0[j] = v.y * qdj; cv1[j] = -v.x * qdj;
        } else {
            v.z += qdj;
            cw0[j] = T(0); cw1[j] = T(0);
            cv0[j] = w.y * qdj; cv1[j] = -w.x * qdj;
        }
        W[j] = w;
        V[j] = v;
        V3<T> In, If;
        inertia_mul(L, w, v, In, If);
        pf[j] = cross(w, If);
        pn[j] = cross_add(cross(w, In), v, If);
    });

    reload_fence();
    ArtI<T> IAc[N];       // articulated inertia accumulators (a parent's, from its children)
    V3<T> pAn[N], pAf[N];  // bias force accumulators
    V3<T> UrD[N], UlD[N];  // U / D (its S-component is exactly 1)
    T uD[N];
    cfor_rev<N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int p = Topo::parent(j);
        constexpr bool pri = Topo::prismatic(j);
        const Link<T> L = load_link(mdl, j);
        ArtI<T> IA;
        V3<T> An, Af;
        if constexpr (Topo::last_child(j) < 0) {  // a leaf: its own rigid inertia
            IA = rigid_inertia(L);
            An = pn[j];
            Af = pf[j];
        } else {
            IA = IAc[j];
            An = pAn[j];
            Af = pAf[j];
        }
        V3<T> ur, ul;
        T D, u;
        if constexpr (!pri) {
            ur = v3(IA.A.xz, IA.A.yz, IA.A.zz);
            ul = v3(IA.B.m[6], IA.B.m[7], IA.B.m[8]);
            D = IA.A.zz;
            u = tv[j] - An.z;
        } else {
            ur = v3(IA.B.m[2], IA.B.m[5], IA.B.m[8]);
            ul = v3(IA.M.xz, IA.M.yz, IA.M.zz);
            D = IA.M.zz;
            u = tv[j] - Af.z;
        }
        const T Dinv = recip(D);
        V3<T> dr = v3(ur.x * Dinv, ur.y * Dinv, ur.z * Dinv);
        V3<T> dl = v3(ul.x * Dinv, ul.y * Dinv, ul.z * Dinv);
        if constexpr (!pri) dr.z = T(1); else dl.z = T(1);
        UrD[j] = dr;
        UlD[j] = dl;
        uD[j] = u * Dinv;
        if constexpr (p >= 0) {
            ArtI<T> Ia;
            Ia.A = S3<T>{fmadd(-ur.x, dr.x, IA.A.xx), fmadd(-ur.x, dr.y, IA.A.xy), fmadd(-ur.x, dr.z, IA.A.xz),
                         fmadd(-ur.y, dr.y, IA.A.yy), fmadd(-ur.y, dr.z, IA.A.yz), fmadd(-ur.z, dr.z, IA.A.zz)};
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const T urr = rr == 0 ? ur.x : (rr == 1 ? ur.y : ur.z);
                Ia.B.m[3 * rr + 0] = fmadd(-urr, dl.x, IA.B.m[3 * rr + 0]);
                Ia.B.m[3 * rr + 1] = fmadd(-urr, dl.y, IA.B.m[3 * rr + 1]);
                Ia.B.m[3 * rr + 2] = fmadd(-urr, dl.z, IA.B.m[3 * rr + 2]);
            }
            Ia.M = S3<T>{fmadd(-ul.x, dl.x, IA.M.xx), fmadd(-ul.x, dl.y, IA.M.xy), fmadd(-ul.x, dl.z, IA.M.xz),
                         fmadd(-ul.y, dl.y, IA.M.yy), fmadd(-ul.y, dl.z, IA.M.yz), fmadd(-ul.z, dl.z, IA.M.zz)};
            if constexpr (!pri) {  // Ia (e_z; 0) = 0: A's z row/column, B's z row
                Ia.A.xz = T(0); Ia.A.yz = T(0); Ia.A.zz = T(0);
                Ia.B.m[6] = T(0); Ia.B.m[7] = T(0); Ia.B.m[8] = T(0);
            } else {  // Ia (0; e_z) = 0: B's z column, M's z row/column
                Ia.B.m[2] = T(0); Ia.B.m[5] = T(0); Ia.B.m[8] = T(0);
                Ia.M.xz = T(0); Ia.M.yz = T(0); Ia.M.zz = T(0);
            }
            // pa = pA + Ia c + U u / D, c = (cw0, cw1, 0; cv0, cv1, 0)
            const V3<T> cr = v3(cw0[j], cw1[j], T(0)), cl = v3(cv0[j], cv1[j], T(0));
            const V3<T> uu = v3(ur.x * uD[j], ur.y * uD[j], ur.z * uD[j]);
            const V3<T> lu = v3(ul.x * uD[j], ul.y * uD[j], ul.z * uD[j]);
            V3<T> pa_n = add3(mul_add(mul_add(An, Ia.A, cr), Ia.B, cl), uu);
            V3<T> pa_f = add3(add3(mul_add(Af, Ia.M, cl), mul_t(Ia.B, cr)), lu);
            M3<T> E;
            V3<T> r;
            link_frame<T, pri>(L, qv[j], cs[j], sn[j], E, r);
            force_to_parent(E, r, pa_n, pa_f);
            const ArtI<T> moved = to_parent(E, r, Ia);
            if constexpr (Topo::last_child(p) == j) {  // first contribution (highest child)
                IAc[p] = moved;
                add_rigid(IAc[p], load_link(mdl, p));
                pAn[p] = add3(pn[p], pa_n);
                pAf[p] = add3(pf[p], pa_f);
            } else {
                add_art(IAc[p], moved);
                pAn[p] = add3(pAn[p], pa_n);
                pAf[p] = add3(pAf[p], pa_f);
            }
        }
    });

    reload_fence();
    V3<T> AW[N], AV[N];
    cfor<0, N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int p = Topo::parent(j);
        constexpr bool pri = Topo::prismatic(j);
        const Link<T> L = load_link(mdl, j);
        M3<T> E;
        V3<T> r;
        link_frame<T, pri>(L, qv[j], cs[j], sn[j], E, r);
        V3<T> aw, av;
        if constexpr (p < 0) {
            const T g = T(kGravity);
            aw = v3(T(0), T(0), T(0));
            av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);
        } else {
            aw = mul_t(E, AW[p]);
            av = mul_t(E, cross_sub(AV[p], r, AW[p]));
        }
        aw.x += cw0[j]; aw.y += cw1[j];
        av.x += cv0[j]; av.y += cv1[j];
        const V3<T> dr = UrD[j], dl = UlD[j];
        const T a = uD[j] - fmadd(dr.x, aw.x, fmadd(dr.y, aw.y, fmadd(dr.z, aw.z,
                                  fmadd(dl.x, av.x, fmadd(dl.y, av.y, dl.z * av.z)))));
        if constexpr (!pri) aw.z += a; else av.z += a;
        AW[j] = aw;
        AV[j] = av;
        out(j, a);
    });
}

// ----------------------------------------------------------------------------- CRBA
// Output as crba_body.hip.hpp: element row + N*col of the column-major matrix, upper
// triangle; strictly-lower entries and non-ancestor pairs exact zeros.
template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void crba_eval_tree(const T *mdl, const T (&qv)[N], Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN upper triangle (spatial.hip.hpp)
    gd.template joints<Topo>(qv);
    auto out = [&](int e, T v) { out_(e, e % N <= e / N ? gd.out(v) : v); };
    T cs[N], sn[N];
    cfor<0, N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (!Topo::prismatic(j)) sin_cos<FAST>(qv[j], sn[j], cs[j]); else { cs[j] = T(1); sn[j] = T(0); }
    });
    ArtI<T> Icc[N];
    cfor_rev<N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int p = Topo::parent(i);
        reload_fence();
        const Link<T> L = load_link(mdl, i);
        ArtI<T> Ic;
        if constexpr (Topo::last_child(i) < 0) Ic = rigid_inertia(L); else Ic = Icc[i];
        // F = Ic S_i
        V3<T> Fn, Ff;
        if constexpr (!Topo::prismatic(i)) {
            Fn = v3(Ic.A.xz, Ic.A.yz, Ic.A.zz);
            Ff = v3(Ic.B.m[6], Ic.B.m[7], Ic.B.m[8]);
        } else {
            Fn = v3(Ic.B.m[2], Ic.B.m[5], Ic.B.m[8]);
            Ff = v3(Ic.M.xz, Ic.M.yz, Ic.M.zz);
        }
        out(i + N * i, Topo::prismatic(i) ? Ff.z : Fn.z);
        cfor<i + 1, N>([&](auto rc) { out(decltype(rc)::value + N * i, T(0)); });
        // carry F up the ancestors: k = i-1 .. 0, transforming across child_on_path(i, k)
        cfor_rev<i>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (Topo::is_ancestor(k, i)) {
                constexpr int c = Topo::child_toward(k, i);
                const Link<T> Lc = load_link(mdl, c);
                M3<T> E;
                V3<T> r;
                link_frame<T, Topo::prismatic(c)>(Lc, qv[c], cs[c], sn[c], E, r);
                force_to_parent(E, r, Fn, Ff);
                out(k + N * i, Topo::prismatic(k) ? Ff.z : Fn.z);
            } else {
                out(k + N * i, T(0));
            }
        });
        if constexpr (p >= 0) {
            M3<T> E;
            V3<T> r;
            link_frame<T, Topo::prismatic(i)>(L, qv[i], cs[i], sn[i], E, r);
            const ArtI<T> moved = to_parent(E, r, Ic);
            if constexpr (Topo::last_child(p) == i) {
                Icc[p] = moved;
                add_rigid(Icc[p], load_link(mdl, p));
            } else {
                add_art(Icc[p], moved);
            }
        }
    });
}

// ------------------------------------------------------------------ FK / Jacobian
// Multibody::fwd_kin (multibody.rs:87-93, translation only, lib.rs:54-55) and ::jac
// (multibody.rs:95-108, body Jacobian of the last link, rows [lin; rot], 6 x N column-major)
// along the last link's ancestor path.
template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void fwd_kin_tree(const T *mdl, const T (&qv)[N], Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<Topo>(qv);
    auto out = [&](int e, T v) { out_(e, gd.out(v)); };
    M3<T> R{{T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1)}};
    V3<T> p = v3(T(0), T(0), T(0));
    cfor<0, N>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (Topo::on_path(j)) {
            const Link<T> L = load_link(mdl, j);
            T c = T(1), s = T(0);
            if constexpr (!Topo::prismatic(j)) sin_cos<FAST>(qv[j], s, c);
            M3<T> E;
            V3<T> r;
            link_frame<T, Topo::prismatic(j)>(L, qv[j], c, s, E, r);
            p = mul_add(p, R, r);
            M3<T> Rn;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    Rn.m[3 * a + b] = fmadd(R.m[3 * a + 0], E.m[b], fmadd(R.m[3 * a + 1], E.m[3 + b], R.m[3 * a + 2] * E.m[6 + b]));
            R = Rn;
        }
    });
    out(0, p.x);
    out(1, p.y);
    out(2, p.z);
}

template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void jac_tree(const T *mdl, const T (&qv)[N], Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<Topo>(qv);
    auto out = [&](int e, T v) { out_(e, gd.out(v)); };
    // acc = pose of the last frame in frame i, leaf -> root, starting from the model tail
    // (the last link's axis-frame change, layout.hpp kTailOut)
    M3<T> R;
#pragma unroll
    for (int k = 0; k < 9; ++k) R.m[k] = mdl[N * kLinkStride + k];
    V3<T> p = v3(T(0), T(0), T(0));
    cfor_rev<N>([&](auto jc) {
        constexpr int i = decltype(jc)::value;
        if constexpr (Topo::on_path(i)) {
            V3<T> lin, rot;
            if constexpr (!Topo::prismatic(i)) {  // S = (e_z, 0): rot = R^T z, lin = R^T (-p x z)
                rot = v3(R.m[6], R.m[7], R.m[8]);
                lin = mul_t(R, v3(-p.y, p.x, T(0)));
            } else {  // S = (0, e_z): lin = R^T z
                rot = v3(T(0), T(0), T(0));
                lin = v3(R.m[6], R.m[7], R.m[8]);
            }
            out(6 * i + 0, lin.x); out(6 * i + 1, lin.y); out(6 * i + 2, lin.z);
            out(6 * i + 3, rot.x); out(6 * i + 4, rot.y); out(6 * i + 5, rot.z);
            const Link<T> L = load_link(mdl, i);
            T c = T(1), s = T(0);
            if constexpr (!Topo::prismatic(i)) sin_cos<FAST>(qv[i], s, c);
            M3<T> E;
            V3<T> r;
            link_frame<T, Topo::prismatic(i)>(L, qv[i], c, s, E, r);
            p = mul_add(r, E, p);  // acc <- T_i acc = (E R, r + E p)
            M3<T> Rn;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    Rn.m[3 * a + b] = fmadd(E.m[3 * a + 0], R.m[b], fmadd(E.m[3 * a + 1], R.m[3 + b], E.m[3 * a + 2] * R.m[6 + b]));
            R = Rn;
        } else {
#pragma unroll
            for (int k = 0; k < 6; ++k) out(6 * i + k, T(0));
        }
    });
}

template <typename T, int N, bool FAST, typename Topo>
__device__ __forceinline__ void fwd_kin_lane_tree(const T *mdl, const T *__restrict__ q, T *__restrict__ pos,
                                                  uint32_t b, int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    fwd_kin_tree<T, N, FAST, Topo>(mdl, qv, [&](int e, T v) { st_row(pos, e * ld, off, v); });
}

template <typename T, int N, bool FAST, typename Topo>
__device__ __forceinline__ void jac_lane_tree(const T *mdl, const T *__restrict__ q, T *__restrict__ J, uint32_t b,
                                              int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    jac_tree<T, N, FAST, Topo>(mdl, qv, [&](int e, T v) { st_row(J, e * ld, off, v); });
}

}  // namespace dev
}  // namespace rbamd
