// rnea_body.hip.hpp -- per-lane RNEA (device).  Shared by the precompiled kernels
// (rnea.hip, model constants staged in LDS) and the model-specialised kernels compiled
// at load time by hipRTC (jit.cpp, model constants as compile-time immediates).
#pragma once

#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

// ----------------------------------------------------------------------------- RNEA
// Per-link steps of the serial-chain RNEA (rnea_eval).
template <typename T>
struct RneaState {
    V3<T> w, v, aw, av;  // link velocity / acceleration (rot, lin), link coordinates
};

// Link 0: v_{-1} = 0, a_{-1} = (0, (0,0,+g)) -- multibody.rs:116-120
// GF (centre-of-mass form only): ff receives g = f / m (spatial.hip.hpp link_force_g).
// Each step checks its link's inputs into gd (InputGuard, spatial.hip.hpp) where it consumes them.
// RB_GUARD_ANCHOR (jit.cpp: rollouts and chains longer than 8 links) also adds the running check
// -- +-0 while every input so far was in range -- to w.z: that use pins each link's check next to
// its work, where the scheduler would otherwise sink the checks towards the stores and keep the
// input rows live across the sweep (30-link fp32 parked RNEA: 151 VGPRs anchored, 168 + 200 B of
// scratch not; fp64 FR3 rollout 127 vs 129, the 4th wave per SIMD).  Short-chain RNEA / FD
// kernels are tighter without it (fp64 FR3 RNEA pair 127 vs 135 VGPRs).
#ifndef RB_GUARD_ANCHOR
#define RB_GUARD_ANCHOR 0
#endif
// QDD = false: qdd is the constant 0 of a bias sweep (fdh_bias), nothing to check (the guard's
// asm FMA would not fold away on it, spatial.hip.hpp InputGuard).
template <typename T, bool FAST, bool GF = false, bool QDD = true>
RB_HD void rnea_fwd0(const T *mdl, T q0, T qd0, T qdd0, RneaState<T> &st, T &sn, T &cs,
                                          V3<T> &fn, V3<T> &ff, InputGuard<T> &gd) {
    const Link<T> L = load_link(mdl, 0);
    gd.angle(q0);
    gd.val(qd0);
    if constexpr (QDD) gd.val(qdd0);
    sin_cos<FAST>(q0, sn, cs);
    const M3<T> E = joint_rotation(L.Rp, cs, sn);
    const T g = T(kGravity);
    st.w = v3(T(0), T(0), RB_GUARD_ANCHOR ? gd.out(qd0) : qd0);
    st.v = v3(T(0), T(0), T(0));
    st.aw = v3(T(0), T(0), qdd0);
    st.av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);  // E^T (0,0,g)
#if RB_COM_FORM
    if constexpr (GF) {
        link_force_g(L, 0, st.w, st.v, st.aw, st.av, fn, ff);
        return;
    }
#endif
    link_force(L, 0, st.w, st.v, st.aw, st.av, fn, ff);  // v = 0 folds away
}

// Link j >= 1: forward sweep step (multibody.rs:122-141).
template <typename T, bool FAST, bool GF = false, bool QDD = true>
RB_HD void rnea_fwd(const T *mdl, int j, T qj, T qdj, T qddj, RneaState<T> &st, T &sn, T &cs,
                                         V3<T> &fn, V3<T> &ff, InputGuard<T> &gd) {
    const Link<T> L = load_link(mdl, j);
    gd.angle(qj);
    gd.val(qdj);
    if constexpr (QDD) gd.val(qddj);
    sin_cos<FAST>(qj, sn, cs);
    const M3<T> E = joint_rotation(L.Rp, cs, sn);
    // SpatialVelocity::transform (spatial.rs:110-116) on v and a
    const V3<T> u = cross_sub(st.v, L.p, st.w);
    const V3<T> ua = cross_sub(st.av, L.p, st.aw);
    V3<T> wn = mul_t(E, st.w), vn = mul_t(E, u);
    V3<T> awn = mul_t(E, st.aw), avn = mul_t(E, ua);
    wn.z += qdj;        // multibody.rs:130
    if constexpr (RB_GUARD_ANCHOR != 0) wn.z = gd.out(wn.z);
    awn.z += qddj;      // multibody.rs:133
    avn.x = fmadd(vn.y, qdj, avn.x);   // multibody.rs:135-138, v x (z qd) unrolled
    avn.y = fmadd(-vn.x, qdj, avn.y);
    awn.x = fmadd(wn.y, qdj, awn.x);
    awn.y = fmadd(-wn.x, qdj, awn.y);
    st.w = wn; st.v = vn; st.aw = awn; st.av = avn;
    // f = I a + v x* (I v)   (multibody.rs:140)
#if RB_COM_FORM
    if constexpr (GF) {
        link_force_g(L, j, st.w, st.v, st.aw, st.av, fn, ff);
        return;
    }
#endif
    link_force(L, j, st.w, st.v, st.aw, st.av, fn, ff);
}

// Backward sweep step: f_{j-1} += X_j^-1 f_j  (multibody.rs:145-150).
template <typename T>
RB_HD void rnea_bwd(const T *mdl, int j, T cj, T sj, const V3<T> &ffj, const V3<T> &fnj,
                                         V3<T> &ffp, V3<T> &fnp) {
    const T *c = mdl + j * kLinkStride;
    const M3<T> Rp{{c[kE0 + 0], c[kE0 + 1], c[kE0 + 2], c[kE0 + 3], c[kE0 + 4], c[kE0 + 5],
                    c[kE0 + 6], c[kE0 + 7], c[kE0 + 8]}};
    const V3<T> p = v3(c[kP + 0], c[kP + 1], c[kP + 2]);
    // E x = R_p (Rz x)
    const V3<T> zf = v3(fmadd(cj, ffj.x, -sj * ffj.y), fmadd(sj, ffj.x, cj * ffj.y), ffj.z);
    const V3<T> zn = v3(fmadd(cj, fnj.x, -sj * fnj.y), fmadd(sj, fnj.x, cj * fnj.y), fnj.z);
    const V3<T> fl = mul(Rp, zf);
    ffp = v3(ffp.x + fl.x, ffp.y + fl.y, ffp.z + fl.z);
    fnp = cross_add(mul_add(fnp, Rp, zn), p, fl);
}

// Backward sweep over link forces left unscaled by the forward sweep (link_force_g: n_j and
// g_j = f_j / m_j), for model-specialised kernels whose R_p are signed permutations
// (RB_SPLIT_ROT) with centre-of-mass link forces: each step forms the parent's transmitted force
// F_{j-1} = m_{j-1} g_{j-1} + E_j F_j and moment n_{j-1} + E_j n_j + p_j x (E_j F_j)
// (multibody.rs:143-150), so the link force's scaling and both accumulations are FMAs with the
// child's terms as addends (E = R_p Rz(q) has two (cos, sin) rows and one +-e_z row).
// tau_j = n_j.z (multibody.rs:144) goes to out(j, value), leaf first.
#if RB_COM_FORM
constexpr bool kRneaGForm = RB_SPLIT_ROT != 0;
#else
constexpr bool kRneaGForm = false;
#endif

template <typename T, int N, typename Out>
RB_HD void rnea_bwd_g(const T *mdl, const T (&cs)[N], const T (&sn)[N], const V3<T> (&fn)[N], const V3<T> (&g)[N],
                      Out &&out) {
    const T ml = load_link(mdl, N - 1).m;
    V3<T> F = v3(ml * g[N - 1].x, ml * g[N - 1].y, ml * g[N - 1].z);
    V3<T> n = fn[N - 1];
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        out(j, n.z);
        const Link<T> L = load_link(mdl, j);
        const M3<T> E = joint_rotation(L.Rp, cs[j], sn[j]);
        const V3<T> fl = mul(E, F);
        const T mp = load_link(mdl, j - 1).m;
        F = v3(fmadd(mp, g[j - 1].x, fl.x), fmadd(mp, g[j - 1].y, fl.y), fmadd(mp, g[j - 1].z, fl.z));
        n = cross_add(mul_add(fn[j - 1], E, n), L.p, fl);
    }
    out(0, n.z);
}

template <typename T>
RB_HD void poison_leaf(const InputGuard<T> &gd, V3<T> &n, V3<T> &f) {
    n = v3(gd.out(n.x), gd.out(n.y), gd.out(n.z));
    f = v3(gd.out(f.x), gd.out(f.y), gd.out(f.z));
}

// Forward sweep (multibody.rs:122-141) then backward sweep (143-150), fused: the
// per-link forces never leave registers.  One call evaluates the configuration whose
// joint values are in (qv, qdv, qddv) and hands tau_j to `out(j, value)`.
template <typename T, int N, bool FAST, typename Out>
RB_HD void rnea_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N],
                                          const T (&qddv)[N], Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN torques (spatial.hip.hpp)
    // short chains poison the n outputs, long ones the leaf's wrench (below)
    constexpr bool kLeaf = N > 8;
    auto out = [&](int j, T v) { out_(j, kLeaf ? v : gd.out(v)); };
    T cs[N], sn[N];
    V3<T> fn[N], ff[N];  // per-link spatial force: moment n (rot), force f (lin) -- or g = f / m
    RneaState<T> st;
    rnea_fwd0<T, FAST, kRneaGForm>(mdl, qv[0], qdv[0], qddv[0], st, sn[0], cs[0], fn[0], ff[0], gd);
#pragma unroll
    for (int j = 1; j < N; ++j)
        rnea_fwd<T, FAST, kRneaGForm>(mdl, j, qv[j], qdv[j], qddv[j], st, sn[j], cs[j], fn[j], ff[j], gd);

    // Long chains: the input check poisons the leaf's wrench; the backward sweep carries a
    // fully-NaN wrench to every parent (each row of E = R_p Rz(q) has an entry that is not a
    // folded zero), so every tau is NaN -- 6 adds where poisoning the outputs takes n.
    if constexpr (kLeaf) poison_leaf(gd, fn[N - 1], ff[N - 1]);
    // Backward sweep: tau_i = n_i.z (multibody.rs:144)
    reload_fence();
    if constexpr (kRneaGForm) {
        rnea_bwd_g<T, N>(mdl, cs, sn, fn, ff, out);
        return;
    }
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        out(j, fn[j].z);
        rnea_bwd(mdl, j, cs[j], sn[j], ff[j], fn[j], ff[j - 1], fn[j - 1]);
    }
    out(0, fn[0].z);
}

template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void rnea_any(const T *mdl, const T (&qv)[N], const T (&qdv)[N], const T (&qddv)[N],
                                         Out &&out) {
    if constexpr (Topo::kSerial)
        rnea_eval<T, N, FAST>(mdl, qv, qdv, qddv, static_cast<Out &&>(out));
    else
        rnea_eval_tree<T, N, FAST, Topo>(mdl, qv, qdv, qddv, static_cast<Out &&>(out));
}

template <typename T, int N>
__device__ __forceinline__ void load_cfg(const T *__restrict__ a, const T *__restrict__ b,
                                         const T *__restrict__ c, int64_t ld, uint32_t off,
                                         T (&x)[N], T (&y)[N], T (&z)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        x[j] = ld_row(a, j * ld, off);
        y[j] = ld_row(b, j * ld, off);
        z[j] = ld_row(c, j * ld, off);
    }
}

// Lane bodies: `mdl` points at the packed model (LDS copy or a constexpr array).
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rnea_lane(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                          const T *__restrict__ qdd, T *__restrict__ tau, uint32_t b,
                                          int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N], qddv[N];
    load_cfg<T, N>(q, qd, qdd, ld, off, qv, qdv, qddv);
    rnea_any<T, N, FAST, Topo>(mdl, qv, qdv, qddv, [&](int j, T v) { st_row(tau, j * ld, off, v); });
}

// Sequential pair (tuning pack=3, A/B): see aba_lane_seq2.
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rnea_lane_seq2(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                               const T *__restrict__ qdd, T *__restrict__ tau, uint32_t offA,
                                               uint32_t offB, bool two, int64_t ld) {
    T qa[N], qda[N], qdda[N], qb[N], qdb[N], qddb[N];
    const uint32_t ob = two ? offB : offA;
    load_cfg<T, N>(q, qd, qdd, ld, offA, qa, qda, qdda);
    load_cfg<T, N>(q, qd, qdd, ld, ob, qb, qdb, qddb);
    rnea_any<T, N, FAST, Topo>(mdl, qa, qda, qdda, [&](int j, T v) { st_row(tau, j * ld, offA, v); });
    if (two) rnea_any<T, N, FAST, Topo>(mdl, qb, qdb, qddb, [&](int j, T v) { st_row(tau, j * ld, offB, v); });
}

// Long serial chains in fp32 (jit rnea_park = NP > 0, model-specialised, centre-of-mass g-form):
// the same arithmetic as rnea_eval with fewer live values, for 3 waves per SIMD where rnea_lane
// holds ~240 (30 links: per link n, g and (cos, sin) -- 246 VGPRs, 2 waves/SIMD).
//   * the first NP links' (n, g) go to LDS during the forward sweep (the backward sweep needs
//     them last): NP x 6 rows x 64 lanes x 4 B per wave (NP = 8: 12 KB, 12 waves per CU);
//   * (cos, sin) are not kept: the backward sweep reloads q_j (a row the lane read moments
//     before -- an L2 / Infinity Cache hit) D links ahead and re-evaluates the same sincos, so
//     every value equals rnea_eval's bit for bit.
template <typename T, int N, bool FAST, int NP>
__device__ __forceinline__ void rnea_lane_park(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                               const T *__restrict__ qdd, T *__restrict__ tau, uint32_t b,
                                               int64_t ld) {
    static_assert(kRneaGForm && NP > 0 && NP < N, "centre-of-mass g-form serial chains only");
    constexpr int D = 4;  // backward-sweep reload distance (links)
    __shared__ T park[4][NP * 6][64];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N], qddv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {  // q temporal: the backward sweep reads it again
        qv[j] = ld_row<T, false>(q, j * ld, off);
        qdv[j] = ld_row(qd, j * ld, off);
        qddv[j] = ld_row(qdd, j * ld, off);
    }
    InputGuard<T> gd;  // out-of-domain configurations: NaN torques (spatial.hip.hpp)
    V3<T> fn[N], gg[N];  // entries j < NP live in LDS after the forward sweep
    auto put = [&](int j) {
        const T v[6] = {fn[j].x, fn[j].y, fn[j].z, gg[j].x, gg[j].y, gg[j].z};
#pragma unroll
        for (int k = 0; k < 6; ++k) park[w][6 * j + k][l] = v[k];
    };
    RneaState<T> st;
    T sn, cs;
    rnea_fwd0<T, FAST, true>(mdl, qv[0], qdv[0], qddv[0], st, sn, cs, fn[0], gg[0], gd);
    put(0);
#pragma unroll
    for (int j = 1; j < N; ++j) {
        rnea_fwd<T, FAST, true>(mdl, j, qv[j], qdv[j], qddv[j], st, sn, cs, fn[j], gg[j], gd);
        if (j < NP) put(j);
    }
    poison_leaf(gd, fn[N - 1], gg[N - 1]);  // as rnea_eval
    reload_fence();
    T qr[N];
#pragma unroll
    for (int j = N - 1; j >= N - D && j >= 1; --j) qr[j] = ld_row<T, false>(q, j * ld, off);
    __builtin_amdgcn_sched_barrier(0);
    // rnea_bwd_g (above) with (cos, sin) from the reloaded q and the first links' forces from LDS
    const T ml = load_link(mdl, N - 1).m;
    V3<T> F = v3(ml * gg[N - 1].x, ml * gg[N - 1].y, ml * gg[N - 1].z);
    V3<T> n = fn[N - 1];
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        st_row(tau, j * ld, off, n.z);
        if (j - D >= 1) qr[j - D] = ld_row<T, false>(q, (j - D) * ld, off);
        T s, c;
        sin_cos<FAST>(qr[j], s, c);
        const Link<T> L = load_link(mdl, j);
        const M3<T> E = joint_rotation(L.Rp, c, s);
        const V3<T> fl = mul(E, F);
        V3<T> fp = fn[j - 1], gp = gg[j - 1];
        if (j - 1 < NP) {
            fp = v3(park[w][6 * (j - 1) + 0][l], park[w][6 * (j - 1) + 1][l], park[w][6 * (j - 1) + 2][l]);
            gp = v3(park[w][6 * (j - 1) + 3][l], park[w][6 * (j - 1) + 4][l], park[w][6 * (j - 1) + 5][l]);
        }
        const T mp = load_link(mdl, j - 1).m;
        F = v3(fmadd(mp, gp.x, fl.x), fmadd(mp, gp.y, fl.y), fmadd(mp, gp.z, fl.z));
        n = cross_add(mul_add(fp, E, n), L.p, fl);
        __builtin_amdgcn_sched_barrier(0);
    }
    st_row(tau, 0, off, n.z);
}

// Reversed-sweep form of long serial chains (fp64; jit.cpp): no per-link storage.  The forward
// sweep (multibody.rs:122-141) carries only the link kinematics (w, v, aw, av) to the leaf; the
// backward sweep (143-150) walks back from the leaf, each step forming link j's wrench from its
// kinematics (link_force_g), adding the child's transmitted wrench, and recovering link j-1's
// kinematics by inverting the forward step with the reloaded q_j and the kept qd_j, qdd_j -- E_j
// is orthonormal, so
//   w_{j-1}  = E (w_j - qd z)                 aw_{j-1} = E (aw_j - qdd z - w_j x qd z)
//   v_{j-1}  = E v_j + p x w_{j-1}            av_{j-1} = E (av_j - v_j x qd z) + p x aw_{j-1}.
// Live set: the 12 kinematic values, the 6 of the transmitted wrench, qd / qdd and the rows in flight,
// where rnea_eval holds (n, g) and (cos, sin) per link (fp64, 30 links: ~500 VGPRs, one wave per
// SIMD; parking them in LDS as rnea_lane_park does would need 60 KB per wave).  The kinematics
// are evaluated twice (once each way), sincos twice, and q is read twice; the recovered
// kinematics carry a few extra roundings per link.
template <typename T, int N, bool FAST>
__device__ __forceinline__ void rnea_lane_rev(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                              const T *__restrict__ qdd, T *__restrict__ tau, uint32_t b,
                                              int64_t ld) {
    static_assert(RB_COM_FORM != 0, "centre-of-mass link forces (link_force_g) only");
    constexpr int PF = 4, PB = 4;  // load distance (links) of the forward / backward sweep
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N], qddv[N];
    auto load = [&](int j) {  // q temporal: the backward sweep reads it again
        qv[j] = ld_row<T, false>(q, j * ld, off);
        qdv[j] = ld_row(qd, j * ld, off);
        qddv[j] = ld_row(qdd, j * ld, off);
    };
#pragma unroll
    for (int j = 0; j < PF && j < N; ++j) load(j);
    InputGuard<T> gd;  // out-of-domain configurations: NaN torques (spatial.hip.hpp)
    RneaState<T> st;
    {  // link 0's kinematics (rnea_fwd0; its wrench is formed in the backward sweep)
        T sn, cs;
        gd.angle(qv[0]);
        gd.val(qdv[0]);
        gd.val(qddv[0]);
        sin_cos<FAST>(qv[0], sn, cs);
        const M3<T> E = joint_rotation(load_link(mdl, 0).Rp, cs, sn);
        const T g = T(kGravity);
        st.w = v3(T(0), T(0), RB_GUARD_ANCHOR ? gd.out(qdv[0]) : qdv[0]);
        st.v = v3(T(0), T(0), T(0));
        st.aw = v3(T(0), T(0), qddv[0]);
        st.av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);
    }
#pragma unroll
    for (int j = 1; j < N; ++j) {
        if (j + PF - 1 < N) load(j + PF - 1);
        const Link<T> L = load_link(mdl, j);
        const T qj = qv[j], qdj = qdv[j], qddj = qddv[j];
        gd.angle(qj);
        gd.val(qdj);
        gd.val(qddj);
        T sn, cs;
        sin_cos<FAST>(qj, sn, cs);
        const M3<T> E = joint_rotation(L.Rp, cs, sn);
        const V3<T> u = cross_sub(st.v, L.p, st.w);
        const V3<T> ua = cross_sub(st.av, L.p, st.aw);
        V3<T> wn = mul_t(E, st.w), vn = mul_t(E, u);
        V3<T> awn = mul_t(E, st.aw), avn = mul_t(E, ua);
        wn.z += qdj;
        if constexpr (RB_GUARD_ANCHOR != 0) wn.z = gd.out(wn.z);
        awn.z += qddj;
        avn.x = fmadd(vn.y, qdj, avn.x);
        avn.y = fmadd(-vn.x, qdj, avn.y);
        awn.x = fmadd(wn.y, qdj, awn.x);
        awn.y = fmadd(-wn.x, qdj, awn.y);
        st.w = wn; st.v = vn; st.aw = awn; st.av = avn;
        __builtin_amdgcn_sched_barrier(0);  // keeps the loads PF links ahead, not all hoisted
    }
    reload_fence();
    // backward sweep: rows reloaded PB links ahead, leaf first
    // qd, qdd stay in registers from the forward sweep; only q is reloaded (30 links fp64: 184
    // registers, 2 waves/SIMD, 227.9 vs 241.0 us tiled and 233.5 vs 258.0 SoA against reloading
    // all three rows at 93 registers / 5 waves, whose reloads reach HBM: 1.61x the bytes)
    auto reload = [&](int j) { qv[j] = ld_row<T, false>(q, j * ld, off); };
#pragma unroll
    for (int j = N - 1; j >= N - PB && j >= 0; --j) reload(j);
    V3<T> F, n;  // the wrench link j transmits to its parent, in link j's frame
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        if (j - PB >= 0) reload(j - PB);
        const Link<T> L = load_link(mdl, j);
        V3<T> fn, gg;
        link_force_g(L, j, st.w, st.v, st.aw, st.av, fn, gg);
        if (j == N - 1) {
            poison_leaf(gd, fn, gg);  // as rnea_eval: a NaN wrench reaches every parent
            F = v3(L.m * gg.x, L.m * gg.y, L.m * gg.z);
            n = fn;
        } else {
            F = v3(fmadd(L.m, gg.x, F.x), fmadd(L.m, gg.y, F.y), fmadd(L.m, gg.z, F.z));
            n = v3(fn.x + n.x, fn.y + n.y, fn.z + n.z);
        }
        st_row(tau, j * ld, off, n.z);
        if (j == 0) break;
        T s, c;
        sin_cos<FAST>(qv[j], s, c);
        const M3<T> E = joint_rotation(L.Rp, c, s);
        const T qdj = qdv[j], qddj = qddv[j];
        const V3<T> fl = mul(E, F);  // the parent's share: E F and E n + p x (E F)
        n = cross_add(mul(E, n), L.p, fl);
        F = fl;
        const V3<T> wp = mul(E, v3(st.w.x, st.w.y, st.w.z - qdj));
        const V3<T> awp = mul(E, v3(fmadd(-st.w.y, qdj, st.aw.x), fmadd(st.w.x, qdj, st.aw.y), st.aw.z - qddj));
        const V3<T> vp = cross_add(mul(E, st.v), L.p, wp);
        const V3<T> avp = cross_add(mul(E, v3(fmadd(-st.v.y, qdj, st.av.x), fmadd(st.v.x, qdj, st.av.y), st.av.z)),
                                    L.p, awp);
        st.w = wp; st.v = vp; st.aw = awp; st.av = avp;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Streaming form (precompiled generic kernels, rnea.hip): walk the batch with `stride`,
// prefetching the next configuration's joint values into registers before evaluating the
// current one.
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rnea_stream_lane(const T *mdl, const T *__restrict__ q,
                                                 const T *__restrict__ qd, const T *__restrict__ qdd,
                                                 T *__restrict__ tau, uint32_t b, uint32_t stride,
                                                 uint32_t B, int64_t ld, T (&qv)[N], T (&qdv)[N],
                                                 T (&qddv)[N]) {
    for (;;) {
        const uint32_t bn = b + stride;
        const bool more = bn < B;
        T nq[N], nqd[N], nqdd[N];
        if (more) load_cfg<T, N>(q, qd, qdd, ld, bn * (uint32_t)sizeof(T), nq, nqd, nqdd);
        const uint32_t off = b * (uint32_t)sizeof(T);
        rnea_any<T, N, FAST, Topo>(mdl, qv, qdv, qddv, [&](int j, T v) { st_row(tau, j * ld, off, v); });
        if (!more) break;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = nq[j];
            qdv[j] = nqd[j];
            qddv[j] = nqdd[j];
        }
        b = bn;
    }
}

}  // namespace dev
}  // namespace rbamd
