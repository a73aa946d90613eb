// aba_body.hip.hpp -- per-lane forward dynamics by the Articulated-Body Algorithm
// (device).  Shared by the precompiled kernels (aba.hip) and the model-specialised
// hipRTC kernels (jit.cpp).  Featherstone Table 7.1 with z-axis joints (S = rot z) and
// the reference's fictitious-gravity base acceleration (0, +g) (multibody.rs:117-120);
// defines qdd = sym(H)^-1 (tau - rnea(q, qd, 0)) with H from Multibody::crba
// (multibody.rs:155-174) -- the reference has no forward-dynamics solve.
#pragma once

#include "fdh_body.hip.hpp"
#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

template <typename T, int N, bool FAST, typename Out>
RB_HD void aba_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N], const T (&tv)[N],
                                         Out &&out_) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN accelerations (spatial.hip.hpp)
    gd.template joints<SerialTopo>(qv);
    gd.vals(qdv);
    gd.vals(tv);
    auto out = [&](int j, T v) { out_(j, gd.out(v)); };
    T cs[N], sn[N];
    T cw0[N], cw1[N], cv0[N], cv1[N];  // c_i = v_i x (S qd_i): (w.y qd, -w.x qd, 0; v.y qd, -v.x qd, 0)
    V3<T> pn[N], pf[N];                // bias force p_i = v_i x* (I_i v_i)

    // Pass 1: velocities and bias terms.
    V3<T> w = v3(T(0), T(0), T(0)), v = v3(T(0), T(0), T(0));
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const Link<T> L = load_link(mdl, j);
        sin_cos<FAST>(qv[j], sn[j], cs[j]);
        const T qdj = qdv[j];
        if (j == 0) {
            w = v3(T(0), T(0), qdj);
            v = v3(T(0), T(0), T(0));
        } else {
            const M3<T> E = joint_rotation(L.Rp, cs[j], sn[j]);
            const V3<T> u = cross_sub(v, L.p, w);
            w = mul_t(E, w);
            v = mul_t(E, u);
            w.z += qdj;
        }
        cw0[j] = w.y * qdj; cw1[j] = -w.x * qdj;
        cv0[j] = v.y * qdj; cv1[j] = -v.x * qdj;
        V3<T> In, If;
        inertia_mul(L, w, v, In, If);
        pf[j] = cross(w, If);
        pn[j] = cross_add(cross(w, In), v, If);
    }

    // Pass 2: articulated inertias, leaf to root.
    reload_fence();
    // Pass-3 state per joint: U/D = (dr.x, dr.y, 1; dl) -- U's own z entry is D -- and u/D.
    T Drx[N], Dry[N], Dl[N][3], uD[N];
    ArtI<T> IA = rigid_inertia(load_link(mdl, N - 1));
    V3<T> pAn = pn[N - 1], pAf = pf[N - 1];
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        const V3<T> ur = v3(IA.A.xz, IA.A.yz, IA.A.zz);
        const V3<T> ul = v3(IA.B.m[6], IA.B.m[7], IA.B.m[8]);
        const T Dinv = recip(IA.A.zz);  // hardware reciprocal (spatial.hip.hpp)
        const T u = tv[j] - pAn.z;
        Drx[j] = ur.x * Dinv; Dry[j] = ur.y * Dinv;
        Dl[j][0] = ul.x * Dinv; Dl[j][1] = ul.y * Dinv; Dl[j][2] = ul.z * Dinv;
        uD[j] = u * Dinv;
        if (j > 0) {
            const V3<T> dr = v3(Drx[j], Dry[j], T(1));
            const V3<T> dl = v3(Dl[j][0], Dl[j][1], Dl[j][2]);
            // Ia = IA - U U^T / D.  Ia S = 0 exactly (S = rot z), so Ia's rot-z row/column
            // (A.xz, A.yz, A.zz and B's z row) are literal zeros; writing them as such lets
            // every later product skip those terms (Featherstone 2008 §7.3).
            ArtI<T> Ia;
            Ia.A = S3<T>{fmadd(-dr.x, ur.x, IA.A.xx), fmadd(-dr.x, ur.y, IA.A.xy), T(0),
                         fmadd(-dr.y, ur.y, IA.A.yy), T(0), T(0)};
            const T drv[3] = {dr.x, dr.y, dr.z};
            const T ulv[3] = {ul.x, ul.y, ul.z};
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) Ia.B.m[3 * r + c] = fmadd(-drv[r], ulv[c], IA.B.m[3 * r + c]);
            Ia.B.m[6] = T(0); Ia.B.m[7] = T(0); Ia.B.m[8] = T(0);
            Ia.M = S3<T>{fmadd(-dl.x, ul.x, IA.M.xx), fmadd(-dl.x, ul.y, IA.M.xy), fmadd(-dl.x, ul.z, IA.M.xz),
                         fmadd(-dl.y, ul.y, IA.M.yy), fmadd(-dl.y, ul.z, IA.M.yz), fmadd(-dl.z, ul.z, IA.M.zz)};
            // pa = pA + Ia c + U u / D,   c = (cw0, cw1, 0; cv0, cv1, 0); S^T pa = tau exactly
            const T a0 = cw0[j], a1 = cw1[j], b0 = cv0[j], b1 = cv1[j];
            V3<T> pa_n = v3(fmadd(Ia.A.xx, a0, fmadd(Ia.A.xy, a1, fmadd(Ia.B.m[0], b0, fmadd(Ia.B.m[1], b1, fmadd(dr.x, u, pAn.x))))),
                            fmadd(Ia.A.xy, a0, fmadd(Ia.A.yy, a1, fmadd(Ia.B.m[3], b0, fmadd(Ia.B.m[4], b1, fmadd(dr.y, u, pAn.y))))),
                            tv[j]);
            V3<T> pa_f = v3(fmadd(Ia.B.m[0], a0, fmadd(Ia.B.m[3], a1, fmadd(Ia.M.xx, b0, fmadd(Ia.M.xy, b1, fmadd(dl.x, u, pAf.x))))),
                            fmadd(Ia.B.m[1], a0, fmadd(Ia.B.m[4], a1, fmadd(Ia.M.xy, b0, fmadd(Ia.M.yy, b1, fmadd(dl.y, u, pAf.y))))),
                            fmadd(Ia.B.m[2], a0, fmadd(Ia.B.m[5], a1, fmadd(Ia.M.xz, b0, fmadd(Ia.M.yz, b1, fmadd(dl.z, u, pAf.z))))));
            // to the parent frame
            const Link<T> L = load_link(mdl, j);
            const M3<T> E = joint_rotation(L.Rp, cs[j], sn[j]);
            const V3<T> fl = mul(E, pa_f);
            const V3<T> nl = cross_add(mul(E, pa_n), L.p, fl);
            pAf = v3(pf[j - 1].x + fl.x, pf[j - 1].y + fl.y, pf[j - 1].z + fl.z);
            pAn = v3(pn[j - 1].x + nl.x, pn[j - 1].y + nl.y, pn[j - 1].z + nl.z);
            if constexpr (RB_SPLIT_ROT != 0)
                IA = to_parent_split(L.Rp, cs[j], sn[j], E, L.p, Ia);
            else
                IA = to_parent(E, L.p, Ia);
            add_rigid(IA, load_link(mdl, j - 1));
        }
    }

    // Pass 3: accelerations, root to leaf.
    reload_fence();
    V3<T> aw = v3(T(0), T(0), T(0)), av = v3(T(0), T(0), T(0));
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const Link<T> L = load_link(mdl, j);
        const M3<T> E = joint_rotation(L.Rp, cs[j], sn[j]);
        if (j == 0) {
            const T g = T(kGravity);
            aw = v3(T(0), T(0), T(0));
            av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);
        } else {
            const V3<T> ua = cross_sub(av, L.p, aw);
            aw = mul_t(E, aw);
            av = mul_t(E, ua);
        }
        aw.x += cw0[j]; aw.y += cw1[j];
        av.x += cv0[j]; av.y += cv1[j];
        const T a = uD[j] - fmadd(Drx[j], aw.x, fmadd(Dry[j], aw.y, fmadd(Dl[j][0], av.x,
                                  fmadd(Dl[j][1], av.y, fmadd(Dl[j][2], av.z, aw.z)))));
        aw.z += a;
        out(j, a);
    }
}

template <typename T, int N, bool FAST, typename Topo, typename Out>
RB_HD void aba_any(const T *mdl, const T (&qv)[N], const T (&qdv)[N], const T (&tv)[N],
                                        Out &&out) {
    if constexpr (Topo::kSerial)
        aba_eval<T, N, FAST>(mdl, qv, qdv, tv, static_cast<Out &&>(out));
    else
        aba_eval_tree<T, N, FAST, Topo>(mdl, qv, qdv, tv, static_cast<Out &&>(out));
}

template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void aba_lane(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                         const T *__restrict__ tau, T *__restrict__ qdd, uint32_t b,
                                         int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N], tv[N];
    // In order of first use: q, qd root->leaf (pass 1), tau leaf->root (pass 2).  A
    // scheduling barrier after each load pins this issue order; loads retire in issue order,
    // so every counted wait releases as soon as its own row has arrived, and all loads are in
    // flight before the first wait.
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row(q, j * ld, off);
        __builtin_amdgcn_sched_barrier(0);
        qdv[j] = ld_row(qd, j * ld, off);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        tv[j] = ld_row(tau, j * ld, off);
        __builtin_amdgcn_sched_barrier(0);
    }
    aba_any<T, N, FAST, Topo>(mdl, qv, qdv, tv, [&](int j, T v) { st_row(qdd, j * ld, off, v); });
}

// Paired lane (fp32 model-specialised kernels, spatial.hip.hpp f2): the configurations at
// byte offsets offA / offB from the pair's base (ld_row2); loads in the same first-use order
// as aba_lane.
template <int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void aba_lane2(const f2 *mdl, const float *__restrict__ q, const float *__restrict__ qd,
                                          const float *__restrict__ tau, float *__restrict__ qdd, uint32_t offA,
                                          uint32_t offB, int64_t ld) {
    f2 qv[N], qdv[N], tv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row2(q, j * ld, offA, offB);
        __builtin_amdgcn_sched_barrier(0);
        qdv[j] = ld_row2(qd, j * ld, offA, offB);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) {
        tv[j] = ld_row2(tau, j * ld, offA, offB);
        __builtin_amdgcn_sched_barrier(0);
    }
    aba_any<f2, N, FAST, Topo>(mdl, qv, qdv, tv, [&](int j, f2 v) { st_row2(qdd, j * ld, offA, offB, v); });
}

// Sequential pair (tuning pack=3, A/B): the configurations at byte offsets offA and offB
// (the second only when `two`) evaluated one after the other from one load burst, so the
// second's rows land while the first computes.
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void aba_lane_seq2(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                              const T *__restrict__ tau, T *__restrict__ qdd, uint32_t offA,
                                              uint32_t offB, bool two, int64_t ld) {
    T qa[N], qda[N], ta[N], qb[N], qdb[N], tb[N];
    const uint32_t ob = two ? offB : offA;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qa[j] = ld_row(q, j * ld, offA);
        qda[j] = ld_row(qd, j * ld, offA);
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) ta[j] = ld_row(tau, j * ld, offA);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qb[j] = ld_row(q, j * ld, ob);
        qdb[j] = ld_row(qd, j * ld, ob);
    }
#pragma unroll
    for (int j = N - 1; j >= 0; --j) tb[j] = ld_row(tau, j * ld, ob);
    aba_any<T, N, FAST, Topo>(mdl, qa, qda, ta, [&](int j, T v) { st_row(qdd, j * ld, offA, v); });
    if (two) aba_any<T, N, FAST, Topo>(mdl, qb, qdb, tb, [&](int j, T v) { st_row(qdd, j * ld, offB, v); });
}

// Forward dynamics inside the fused rollout: the mass-matrix form (fdh_body.hip.hpp) when
// RB_ROLLOUT_FDH is set (jit.cpp: serial chains the fd_form policy gives it), else the ABA.
// load_tau(tv) fills the step's torques: for the mass-matrix form after its bias sweep.
#ifndef RB_ROLLOUT_FDH
#define RB_ROLLOUT_FDH 0
#endif
template <typename T, int N, bool FAST, typename Topo, typename Tau, typename Out>
RB_HD void rollout_fd(const T *mdl, const T (&qv)[N], const T (&qdv)[N], Tau &&load_tau, Out &&out) {
    if constexpr (RB_ROLLOUT_FDH != 0 && Topo::kSerial) {
        fdh_eval<T, N, FAST>(mdl, qv, qdv, static_cast<Tau &&>(load_tau), static_cast<Out &&>(out));
    } else {
        T tv[N];
        load_tau(tv);
        aba_any<T, N, FAST, Topo>(mdl, qv, qdv, tv, static_cast<Out &&>(out));
    }
}

// Fused rollout (the MPC-shooting use of forward dynamics): K steps
// of semi-implicit Euler, qd += dt * fd(q, qd, tau_k); q += dt * qd.  q, qd [n][ld] are
// read once and overwritten with the final state; tau_seq is [K][n][ld]; traj
// ([K][n][ld], optional) receives q after each step.
//
// Between steps the state lives in LDS (2N values per lane, row-strided by the block so
// lanes hit distinct banks) when that fits 32 KiB per block: the dynamics already need
// ~110 VGPRs in fp32, and holding q, qd in registers across the K loop on top of them
// costs a wave per SIMD.  Larger chains keep the state in registers.
constexpr int kRolloutBlock = 256;
#ifndef RB_ROLLOUT_NO_HOIST
#define RB_ROLLOUT_NO_HOIST 0
#endif

template <typename T, int N>
constexpr bool rollout_lds_state() {
    return 2 * N * (int)sizeof(T) * kRolloutBlock <= 32768;
}

template <typename T, int N>
struct RolloutShared {
    T x[rollout_lds_state<T, N>() ? 2 * N * kRolloutBlock : 1];
};

template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rollout_lane(const T *mdl, T *__restrict__ q, T *__restrict__ qd,
                                             const T *__restrict__ tau_seq, T dt, int K, T *__restrict__ traj,
                                             uint32_t b, int64_t ld, RolloutShared<T, N> &sh) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    if constexpr (rollout_lds_state<T, N>()) {
        T *sx = sh.x + threadIdx.x;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            sx[j * kRolloutBlock] = ld_row(q, j * ld, off);
            sx[(N + j) * kRolloutBlock] = ld_row(qd, j * ld, off);
        }
        for (int k = 0; k < K; ++k) {
            int64_t ldk = ld;  // RB_ROLLOUT_NO_HOIST (jit.cpp): row offsets re-derived per step
            if constexpr (RB_ROLLOUT_NO_HOIST != 0) asm volatile("" : "+s"(ldk));
            T qv[N], qdv[N];
#pragma unroll
            for (int j = 0; j < N; ++j) {
                qv[j] = sx[j * kRolloutBlock];
                qdv[j] = sx[(N + j) * kRolloutBlock];
            }
            auto load_tau = [&](T (&tv)[N]) {
#pragma unroll
                for (int j = 0; j < N; ++j) tv[j] = ld_row(tau_seq, ((int64_t)k * N + j) * ldk, off);
            };
            // both forms fence memory before their last sweep, so these re-read LDS.
            rollout_fd<T, N, FAST, Topo>(mdl, qv, qdv, load_tau, [&](int j, T a) {
                const T qdn = fmadd(dt, a, sx[(N + j) * kRolloutBlock]);
                const T qn = fmadd(dt, qdn, sx[j * kRolloutBlock]);
                sx[(N + j) * kRolloutBlock] = qdn;
                sx[j * kRolloutBlock] = qn;
                if (traj) st_row(traj, ((int64_t)k * N + j) * ldk, off, qn);
            });
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            st_row(q, j * ld, off, sx[j * kRolloutBlock]);
            st_row(qd, j * ld, off, sx[(N + j) * kRolloutBlock]);
        }
    } else {
        T qv[N], qdv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q, j * ld, off);
            qdv[j] = ld_row(qd, j * ld, off);
        }
        for (int k = 0; k < K; ++k) {
            T a[N];
            auto load_tau = [&](T (&tv)[N]) {
#pragma unroll
                for (int j = 0; j < N; ++j) tv[j] = ld_row(tau_seq, ((int64_t)k * N + j) * ld, off);
            };
            rollout_fd<T, N, FAST, Topo>(mdl, qv, qdv, load_tau, [&](int j, T v) { a[j] = v; });
#pragma unroll
            for (int j = 0; j < N; ++j) {
                qdv[j] = fmadd(dt, a[j], qdv[j]);
                qv[j] = fmadd(dt, qdv[j], qv[j]);
            }
            if (traj) {
#pragma unroll
                for (int j = 0; j < N; ++j) st_row(traj, ((int64_t)k * N + j) * ld, off, qv[j]);
            }
        }
        // Recompute the row addresses after the loop rather than holding 2N 64-bit
        // pointers from the loads across all K steps.
        uint32_t off2 = off;
        asm volatile("" : "+v"(off2));
#pragma unroll
        for (int j = 0; j < N; ++j) {
            st_row(q, j * ld, off2, qv[j]);
            st_row(qd, j * ld, off2, qdv[j]);
        }
    }
}

// Paired rollout (fp32 model-specialised kernels, pack 2): the configurations at byte offsets
// offA / offB of the SoA rows (spatial.hip.hpp f2 lanes, as aba_lane2), both states in LDS
// between steps as f2 pairs, row-strided by the block.
template <int N>
struct RolloutShared2 {
    f2 x[2 * N * kRolloutBlock];
};

template <int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rollout_lane2(const f2 *mdl, float *__restrict__ q, float *__restrict__ qd,
                                              const float *__restrict__ tau_seq, float dt, int K,
                                              float *__restrict__ traj, uint32_t offA, uint32_t offB, int64_t ld,
                                              RolloutShared2<N> &sh) {
    f2 *sx = sh.x + threadIdx.x;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        sx[j * kRolloutBlock] = ld_row2(q, j * ld, offA, offB);
        sx[(N + j) * kRolloutBlock] = ld_row2(qd, j * ld, offA, offB);
    }
    const f2 dt2 = f2{dt, dt};
    for (int k = 0; k < K; ++k) {
        // row offsets re-derived per step (scalar ALU): hoisted out of the K loop they would
        // hold 2N 64-bit values in SGPRs, spilled to VGPRs, across every step
        int64_t ldk = ld;
        asm volatile("" : "+s"(ldk));
        f2 qv[N], qdv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = sx[j * kRolloutBlock];
            qdv[j] = sx[(N + j) * kRolloutBlock];
        }
        auto load_tau = [&](f2 (&tv)[N]) {
#pragma unroll
            for (int j = 0; j < N; ++j) tv[j] = ld_row2(tau_seq, ((int64_t)k * N + j) * ldk, offA, offB);
        };
        rollout_fd<f2, N, FAST, Topo>(mdl, qv, qdv, load_tau, [&](int j, f2 a) {
            const f2 qdn = fmadd(dt2, a, sx[(N + j) * kRolloutBlock]);
            const f2 qn = fmadd(dt2, qdn, sx[j * kRolloutBlock]);
            sx[(N + j) * kRolloutBlock] = qdn;
            sx[j * kRolloutBlock] = qn;
            if (traj) st_row2(traj, ((int64_t)k * N + j) * ldk, offA, offB, qn);
        });
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
        st_row2(q, j * ld, offA, offB, sx[j * kRolloutBlock]);
        st_row2(qd, j * ld, offA, offB, sx[(N + j) * kRolloutBlock]);
    }
}

// Split rollout for small batches (jit pack 4, fp32 mass-matrix form; capi.cpp takes it below
// 2^17 configurations): each Euler step is one forward dynamics, split over a pair of packed
// waves as fdh_split_block2 splits one launch -- the bias wave evaluates C(q, qd) for 128
// configurations, the mass wave H, L D L^T, then (block barrier A) the solve and the Euler
// update of the state, which lives in LDS for both; block barrier B hands the new state to the
// bias wave's next step.  Lanes past B compute on the tile's last configuration and store
// nothing; every wave reaches both barriers K times.
template <int N, bool FAST>
__device__ __forceinline__ void rollout_split_block2(const f2 *mdl, float *__restrict__ q, float *__restrict__ qd,
                                                     const float *__restrict__ tau_seq, float dt, int K,
                                                     float *__restrict__ traj, uint32_t B, int64_t ld) {
    __shared__ f2 shX[2][2 * N][64];  // per wave pair: q rows then qd rows, one f2 per lane
    __shared__ f2 shC[2][N][64];
    const uint32_t w = threadIdx.x >> 6, g = w & 1u, l = threadIdx.x & 63u;
    const uint32_t first = blockIdx.x * 256u;  // < B: the grid is ceil(B / 256) blocks
    const uint32_t cA = (g << 7) + l, cB = cA + 64u, last = B - 1u - first;
    const bool liveA = cA <= last, liveB = cB <= last;
    const uint32_t offA = (first + (liveA ? cA : last)) * 4u;
    const uint32_t offB = liveB ? (first + cB) * 4u : offA;
    f2(&sx)[2 * N][64] = shX[g];
    const f2 dt2 = f2{dt, dt};
    if (w < 2) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            sx[j][l] = ld_row2(q, j * ld, offA, offB);
            sx[N + j][l] = ld_row2(qd, j * ld, offA, offB);
        }
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) {
        int64_t ldk = ld;  // row offsets re-derived per step (as rollout_lane2)
        asm volatile("" : "+s"(ldk));
        if (w < 2) {
            f2 qv[N], qdv[N], cs[N], sn[N], C[N];
#pragma unroll
            for (int j = 0; j < N; ++j) {
                qv[j] = sx[j][l];
                qdv[j] = sx[N + j][l];
            }
            InputGuard<f2> gd;  // the state's domain, every step (fdh_split_block2)
            fdh_bias<f2, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
#pragma unroll
            for (int j = 0; j < N; ++j) shC[g][j][l] = gd.out(C[j]);
            __syncthreads();  // A
            __syncthreads();  // B
        } else {
            f2 qv[N], tv[N], cs[N], sn[N], C[N], H[N][N], Di[N];
#pragma unroll
            for (int j = 0; j < N; ++j) tv[j] = ld_row2(tau_seq, ((int64_t)k * N + j) * ldk, offA, offB);
#pragma unroll
            for (int j = 0; j < N; ++j) {
                qv[j] = sx[j][l];
                sin_cos<FAST>(qv[j], sn[j], cs[j]);
            }
            fdh_factor<f2, N>(mdl, cs, sn, H, Di);
            // keep the loads and the factorisation above barrier A (fdh_split_block2)
#pragma unroll
            for (int j = 0; j < N; ++j) {
                asm volatile("" : "+v"(Di[j].x), "+v"(Di[j].y));
                asm volatile("" : "+v"(tv[j].x), "+v"(tv[j].y));
            }
            __syncthreads();  // A
#pragma unroll
            for (int j = 0; j < N; ++j) C[j] = shC[g][j][l];
            InputGuard<f2> gd;
            gd.vals(tv);
            fdh_solve<f2, N>(H, Di, tv, C, [&](int j, f2 a) {
                const f2 qdn = fmadd(dt2, gd.out(a), sx[N + j][l]);
                const f2 qn = fmadd(dt2, qdn, sx[j][l]);
                sx[N + j][l] = qdn;
                sx[j][l] = qn;
                if (traj && liveA) st_row2(traj, ((int64_t)k * N + j) * ldk, offA, offB, qn);
            });
            __syncthreads();  // B
        }
    }
    if (w >= 2 && liveA) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            st_row2(q, j * ld, offA, offB, sx[j][l]);
            st_row2(qd, j * ld, offA, offB, sx[N + j][l]);
        }
    }
}

}  // namespace dev
}  // namespace rbamd
