// fdh_body.hip.hpp -- per-lane forward dynamics by the mass-matrix method (device).
//
// The reference has no forward-dynamics solve; SURVEY §8(a) A10 defines it as
//     qdd = sym(H)^-1 (tau - rnea(q, qd, 0))
// with H from Multibody::crba (multibody.rs:155-174) and the bias torques from
// Multibody::rnea (multibody.rs:111-153) at zero joint acceleration.  This lane body
// evaluates exactly that definition, fused in registers:
//   1. bias torques C = rnea(q, qd, 0): the RNEA sweeps of rnea_body.hip.hpp with qdd = 0
//      (the fictitious-gravity base acceleration, multibody.rs:117-120, stays);
//   2. H by composite rigid bodies (crba_body.hip.hpp crba_core) on the same (cos, sin);
//   3. H = L D L^T (unit lower L, no square roots) and two triangular solves on tau - C.
// Against the Articulated-Body form (aba_body.hip.hpp) it carries far less per-lane state
// across its sweeps -- no per-link articulated inertias or pass-3 projections, the peak is
// the n(n+1)/2 entries of H -- so short chains run at 2-3x the ABA's waves per SIMD; its
// mass-matrix stage grows as n^2, so long chains keep the ABA (jit.cpp jit_fd_form).
//
// Order of work follows the order the rows land: q, qd root->leaf first (the bias sweep's
// first-use order), tau only after that sweep -- it enters at the final solve.
#pragma once

#include "crba_body.hip.hpp"
#include "rnea_body.hip.hpp"

namespace rbamd {
namespace dev {

// Where the tau rows are loaded: 1 = after the bias sweep (default), 0 = with q and qd at the
// start, 2 = after the factorisation (jit_variant bits 0-1 = 1 / 2 select 0 / 2, A/B only).
// After the bias sweep the rows are not held across it (fp64: 121 instead of 134 VGPRs, 4
// waves/SIMD instead of 3) and still land under the mass-matrix stage: FR3 2^20 tiled, fp64
// 56.2 vs 57.0 us, fp32 paired 27.1 vs 28.1 us; at 65536 (fp32) 4.52 vs 4.63 us, while loading
// after the mass matrix exposes the latency there (4.90 us).
#ifndef RB_FDH_TAU_AT
#define RB_FDH_TAU_AT ((RB_VARIANT & 3) == 1 ? 0 : (RB_VARIANT & 3) == 2 ? 2 : 1)
#endif

// 1. bias torques C = rnea(q, qd, 0) (multibody.rs:111-153 with ddq = 0); also the joint
// (cos, sin) the later stages reuse.  Model-specialised kernels with signed-permutation R_p and
// centre-of-mass link forces take the fused backward sweep (rnea_body.hip.hpp rnea_bwd_g: the
// link force's mass scaling and the child accumulations as FMAs; FR3 fp64 5 fewer VALU per link).
// gd: the input check of q and qd (rnea_fwd, InputGuard).
template <typename T, int N, bool FAST>
RB_HD void fdh_bias(const T *mdl, const T (&qv)[N], const T (&qdv)[N], T (&cs)[N], T (&sn)[N], T (&C)[N],
                    InputGuard<T> &gd) {
    V3<T> fn[N], ff[N];  // ff: the link force, or g = f / m (kRneaGForm)
    RneaState<T> st;
    rnea_fwd0<T, FAST, kRneaGForm, false>(mdl, qv[0], qdv[0], T(0), st, sn[0], cs[0], fn[0], ff[0], gd);
#pragma unroll
    for (int j = 1; j < N; ++j)
        rnea_fwd<T, FAST, kRneaGForm, false>(mdl, j, qv[j], qdv[j], T(0), st, sn[j], cs[j], fn[j], ff[j], gd);
    reload_fence();
    RB_STAGE("bias_bwd");
    if constexpr (kRneaGForm) {
        rnea_bwd_g<T, N>(mdl, cs, sn, fn, ff, [&](int j, T v) { C[j] = v; });
    } else {
#pragma unroll
        for (int j = N - 1; j >= 1; --j) {
            C[j] = fn[j].z;
            rnea_bwd(mdl, j, cs[j], sn[j], ff[j], fn[j], ff[j - 1], fn[j - 1]);
        }
        C[0] = fn[0].z;
    }
}

// 3. H = L D L^T in place, root first: L[i][j] (i > j) overwrites H[j][i]; Di = 1 / D.
// Row j's entries are kept unscaled, U[j][i] = L[i][j] D[j], until row i scales them: the
// row starts by turning its column of U into L (L[j][k] = U[k][j] / D[k]), then
//   D[j] = H[j][j] - sum_k L[j][k] U[k][j],   U[j][i] = H[j][i] - sum_k L[j][k] U[k][i]  (i > j)
// -- one multiply per strictly-upper entry (n(n-1)/2) where scaling at the end of the row and
// rebuilding L D at the next needs two.
template <typename T, int N>
RB_HD void fdh_ldl(T (&H)[N][N], T (&Di)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        T d = H[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) {
            const T u = H[k][j];
            const T l = u * Di[k];
            d = fmadd(-l, u, d);
            H[k][j] = l;
        }
        Di[j] = recip(d);
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            T s = H[j][i];
#pragma unroll
            for (int k = 0; k < j; ++k) s = fmadd(-H[k][j], H[k][i], s);
            H[j][i] = s;
        }
    }
}

// 2.-3. the joint-space inertia H (crba_core, upper triangle H[j][i], j <= i, of the ABI's
// column-major matrix), then its factorisation.
template <typename T, int N>
RB_HD void fdh_factor(const T *mdl, const T (&cs)[N], const T (&sn)[N], T (&H)[N][N], T (&Di)[N]) {
    reload_fence();
    RB_STAGE("crba");
    crba_core<T, N>(mdl, cs, sn, [&](int e, T v) {
        const int j = e % N, i = e / N;
        if (j <= i) H[j][i] = v;
    });
    RB_STAGE("ldl");
    fdh_ldl<T, N>(H, Di);
}

// 4. L y = tau - C,  z = D^-1 y,  L^T x = z  (x = qdd); out(j, qdd_j), leaf first.
template <typename T, int N, typename Out>
RB_HD void fdh_solve(const T (&H)[N][N], const T (&Di)[N], const T (&tv)[N], const T (&C)[N], Out &&out) {
    T x[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        T y = tv[i] - C[i];
#pragma unroll
        for (int k = 0; k < i; ++k) y = fmadd(-H[k][i], x[k], y);
        x[i] = y;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        T z = x[i] * Di[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) z = fmadd(-H[i][k], x[k], z);
        x[i] = z;
        out(i, z);
    }
}

template <typename T, int N, bool FAST, typename Tau, typename Out>
RB_HD void fdh_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N], Tau &&load_tau, Out &&out) {
    T cs[N], sn[N], C[N], tv[N], H[N][N], Di[N];
    InputGuard<T> gd;  // out-of-domain configurations: NaN accelerations (spatial.hip.hpp)
    if constexpr (RB_FDH_TAU_AT == 0) load_tau(tv);
    RB_STAGE("bias_fwd");
    fdh_bias<T, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
    if constexpr (RB_FDH_TAU_AT == 1) load_tau(tv);
    fdh_factor<T, N>(mdl, cs, sn, H, Di);
    if constexpr (RB_FDH_TAU_AT >= 2) load_tau(tv);
    gd.vals(tv);
    RB_STAGE("solve");
    fdh_solve<T, N>(H, Di, tv, C, [&](int j, T v) { out(j, gd.out(v)); });
}

// Inverse AND forward dynamics of one (q, qd) from one set of factors (SURVEY §8(d) config 4's
// RNEA + forward-dynamics pair; one launch):
//   tau  = rnea(q, qd, qdd)                       (multibody.rs:111-153)
//   qdd' = sym(H)^-1 (tau_in - rnea(q, qd, 0))    (the A10 definition above)
// The RNEA is affine in qdd with slope H (multibody.rs:155-174 computes that H), so
//   rnea(q, qd, qdd) = C + sym(H) qdd,   C = rnea(q, qd, 0)
// and the pair shares everything but n^2 FMAs: the bias sweep C and (cos, sin) once, H once,
// then the factorisation and the solve on tau_in.  Against an RNEA launch followed by a
// forward-dynamics launch: q and qd are read once (6 n s bytes per configuration instead of
// 8 n s) and the RNEA's own forward sweep with qdd is replaced by the n^2 products.
// Input checks: tau's outputs on (q, qd, qdd), qdd''s on (q, qd, tau_in).

// h = sym(H) qdd from the upper triangle H[j][i] (j <= i) before L D L^T overwrites it, in a
// fixed order (column i from the leaf, its diagonal first, then the rows toward the root) that
// every grid form of the pair shares -- tau = C + h is then bit-identical across them.
template <typename T, int N>
RB_HD void fdh_hq(const T (&H)[N][N], const T (&av)[N], T (&h)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) h[j] = T(0);
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        h[i] = fmadd(H[i][i], av[i], h[i]);
#pragma unroll
        for (int j = i - 1; j >= 0; --j) {
            h[j] = fmadd(H[j][i], av[i], h[j]);
            h[i] = fmadd(H[j][i], av[j], h[i]);
        }
    }
}

template <typename T, int N, bool FAST, typename LoadQdd, typename LoadTau, typename OutTau, typename OutQdd>
RB_HD void fdh_idfd_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N], LoadQdd &&load_qdd, LoadTau &&load_tau,
                         OutTau &&out_tau, OutQdd &&out_qdd) {
    T cs[N], sn[N], C[N], av[N], tv[N], h[N], H[N][N], Di[N];
    InputGuard<T> gd;
    RB_STAGE("bias_fwd");
    fdh_bias<T, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
    load_qdd(av);
    reload_fence();
    RB_STAGE("crba");
    crba_core<T, N>(mdl, cs, sn, [&](int e, T v) {
        const int j = e % N, i = e / N;
        if (j <= i) H[j][i] = v;
    });
    load_tau(tv);
    RB_STAGE("id");
    fdh_hq<T, N>(H, av, h);
    InputGuard<T> gr = gd;  // tau: q, qd, qdd
    gr.vals(av);
#pragma unroll
    for (int j = N - 1; j >= 0; --j) out_tau(j, gr.out(C[j] + h[j]));
    RB_STAGE("ldl");
    fdh_ldl<T, N>(H, Di);
    InputGuard<T> gf = gd;  // qdd': q, qd, tau_in
    gf.vals(tv);
    RB_STAGE("solve");
    fdh_solve<T, N>(H, Di, tv, C, [&](int j, T v) { out_qdd(j, gf.out(v)); });
}

// Lane body of the pair: q, qd rows in first-use order, qdd after the bias sweep, tau_in after
// the mass matrix (it enters at the solve).
template <typename T, int N, bool FAST>
__device__ __forceinline__ void idfd_lane(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                          const T *__restrict__ qdd, const T *__restrict__ tau_in,
                                          T *__restrict__ tau, T *__restrict__ qdd_out, uint32_t b, int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row(q, j * ld, off);
        __builtin_amdgcn_sched_barrier(0);
        qdv[j] = ld_row(qd, j * ld, off);
        __builtin_amdgcn_sched_barrier(0);
    }
    auto rows = [&](const T *__restrict__ src, T (&v)[N]) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            v[j] = ld_row(src, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    fdh_idfd_eval<T, N, FAST>(
        mdl, qv, qdv, [&](T (&v)[N]) { rows(qdd, v); }, [&](T (&v)[N]) { rows(tau_in, v); },
        [&](int j, T v) { st_row(tau, j * ld, off, v); }, [&](int j, T v) { st_row(qdd_out, j * ld, off, v); });
}

// The pair split over two waves (jit pack 5, small batches: at 2^17 configurations the
// one-per-lane grid is 2 waves per SIMD and the launch time is one wave's ~1170-instruction
// stream), as fdh_split_block1 below: per 64 configurations the bias wave evaluates C and the
// q, qd checks and hands both over through LDS; its partner builds H, h = sym(H) qdd and
// L D L^T, then after one block barrier stores tau = C + h and solves.  Same arithmetic as
// idfd_lane (bit-identical outputs), ~620 / ~600 instructions per wave.
template <typename T, int N, bool FAST>
__device__ __forceinline__ void idfd_split_block1(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                                  const T *__restrict__ qdd, const T *__restrict__ tau_in,
                                                  T *__restrict__ tau, T *__restrict__ qdd_out, uint32_t B,
                                                  int64_t ld, int64_t bs) {
    __shared__ T shC[2][N][64];
    __shared__ float shG[2][64];  // the bias wave's running input check (InputGuard acc)
    const uint32_t wr = threadIdx.x >> 6;  // roles alternate as in fdh_split_block1
    const uint32_t w = (((wr ^ blockIdx.x) & 1u) << 1) + (wr >> 1);
    const uint32_t g = w & 1u, l = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x >> 1, first = blockIdx.x * 128u;  // < B (grid ceil(B / 128))
    const uint32_t c = ((blockIdx.x & 1u) << 7) + (g << 6) + l;       // within the tile
    const uint32_t last = B - 1u - tile * 256u;
    const bool live = first + (g << 6) + l < B;
    const uint32_t off = (live ? c : last) * (uint32_t)sizeof(T);
    const int64_t o = (int64_t)tile * bs;
    if (w < 2) {
        T qv[N], qdv[N], cs[N], sn[N], C[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
            qdv[j] = ld_row(qd + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
        InputGuard<T> gd;
        fdh_bias<T, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
#pragma unroll
        for (int j = 0; j < N; ++j) shC[g][j][l] = C[j];
        shG[g][l] = gd.acc;
        __syncthreads();
    } else {
        T qv[N], av[N], tv[N], cs[N], sn[N], C[N], h[N], H[N][N], Di[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            av[j] = ld_row(qdd + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) sin_cos<FAST>(qv[j], sn[j], cs[j]);
        crba_core<T, N>(mdl, cs, sn, [&](int e, T v) {
            const int j = e % N, i = e / N;
            if (j <= i) H[j][i] = v;
        });
        fdh_hq<T, N>(H, av, h);  // qdd's rows die here, before tau_in's land
        InputGuard<T> gr;         // qdd here, q and qd from the bias wave below
        gr.vals(av);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            tv[j] = ld_row(tau_in + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
        fdh_ldl<T, N>(H, Di);
        // everything above feeds only the live-guarded stores: pinned, so the compiler cannot sink
        // it past the barrier (fdh_split_block2)
#pragma unroll
        for (int j = 0; j < N; ++j) {
            asm volatile("" : "+v"(Di[j]));
            asm volatile("" : "+v"(tv[j]));
            asm volatile("" : "+v"(h[j]));
        }
        InputGuard<T> gf;
        gf.vals(tv);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; ++j) C[j] = shC[g][j][l];
        const float gb = shG[g][l];
        gr.acc = guard_add(gr.acc, gb);
        gf.acc = guard_add(gf.acc, gb);
#pragma unroll
        for (int j = N - 1; j >= 0; --j)
            if (live) st_row(tau + o, j * ld, off, gr.out(C[j] + h[j]));
        fdh_solve<T, N>(H, Di, tv, C, [&](int j, T v) {
            if (live) st_row(qdd_out + o, j * ld, off, gf.out(v));
        });
    }
}

// Kinematic trees (Topo, tree_body.hip.hpp): the same definition with the tree forms of its
// stages -- bias torques by rnea_eval_tree at qdd = 0, H by crba_eval_tree (exact zeros for
// joint pairs that are not ancestor / descendant), then the same L D L^T and solves.  Each stage
// evaluates its own (cos, sin) and input checks (an out-of-domain q / qd poisons C and H, tau
// the outputs).
template <typename T, int N, bool FAST, typename Topo, typename Tau, typename Out>
RB_HD void fdh_eval_tree(const T *mdl, const T (&qv)[N], const T (&qdv)[N], Tau &&load_tau, Out &&out) {
    T C[N], tv[N], H[N][N], Di[N], zero[N];
#pragma unroll
    for (int j = 0; j < N; ++j) zero[j] = T(0);
    rnea_eval_tree<T, N, FAST, Topo>(mdl, qv, qdv, zero, [&](int j, T v) { C[j] = v; });
    load_tau(tv);
    reload_fence();
    crba_eval_tree<T, N, FAST, Topo>(mdl, qv, [&](int e, T v) {
        const int j = e % N, i = e / N;
        if (j <= i) H[j][i] = v;
    });
    fdh_ldl<T, N>(H, Di);
    InputGuard<T> gd;
    gd.vals(tv);
    fdh_solve<T, N>(H, Di, tv, C, [&](int j, T v) { out(j, gd.out(v)); });
}

// Lane body: loads in first-use order (q, qd root->leaf, then tau), as aba_lane.
// Decomposition variants (jit_variant, A/B only): bit 2 = no input loads (inputs synthesised
// from the lane index: compute + stores), bit 3 = no dynamics (loads + stores of their sum).
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void fdh_lane(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                         const T *__restrict__ tau, T *__restrict__ qdd, uint32_t b, int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N], qdv[N];
    if constexpr ((RB_VARIANT & 4) != 0) {
        const T x = T((b + blockIdx.x) & 1023u) * T(1e-3);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = x + T(0.1) * T(j) - T(0.5);
            qdv[j] = T(0.7) - x - T(0.05) * T(j);
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
            qdv[j] = ld_row(qd, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    auto load_tau = [&](T (&tv)[N]) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if constexpr ((RB_VARIANT & 4) != 0) {
                tv[j] = qv[N - 1 - j] * T(3);
            } else {
                tv[j] = ld_row(tau, j * ld, off);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    if constexpr ((RB_VARIANT & 8) != 0) {
        T tv[N];
        load_tau(tv);
#pragma unroll
        for (int j = 0; j < N; ++j) st_row(qdd, j * ld, off, qv[j] + qdv[j] + tv[j]);
    } else {
        if constexpr (Topo::kSerial)
            fdh_eval<T, N, FAST>(mdl, qv, qdv, load_tau, [&](int j, T v) { st_row(qdd, j * ld, off, v); });
        else
            fdh_eval_tree<T, N, FAST, Topo>(mdl, qv, qdv, load_tau, [&](int j, T v) { st_row(qdd, j * ld, off, v); });
    }
}

// Paired lane (packed fp32, spatial.hip.hpp f2), as aba_lane2.
template <int N, bool FAST>
__device__ __forceinline__ void fdh_lane2(const f2 *mdl, const float *__restrict__ q, const float *__restrict__ qd,
                                          const float *__restrict__ tau, float *__restrict__ qdd, uint32_t offA,
                                          uint32_t offB, int64_t ld) {
    f2 qv[N], qdv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row2(q, j * ld, offA, offB);
        __builtin_amdgcn_sched_barrier(0);
        qdv[j] = ld_row2(qd, j * ld, offA, offB);
        __builtin_amdgcn_sched_barrier(0);
    }
    fdh_eval<f2, N, FAST>(
        mdl, qv, qdv,
        [&](f2 (&tv)[N]) {
#pragma unroll
            for (int j = 0; j < N; ++j) {
                tv[j] = ld_row2(tau, j * ld, offA, offB);
                __builtin_amdgcn_sched_barrier(0);
            }
        },
        [&](int j, f2 v) { st_row2(qdd, j * ld, offA, offB, v); });
}

// Small batches on packed lanes (jit pack 4, fp32; the rollout's split, and fp32 FD by tuning
// -- capi.cpp fd_pack takes pack 5 up to 2^17 configurations).  There the one-per-lane grid is at most one wave per SIMD and the kernel
// time is the load burst plus ONE wave's dependent instruction stream (~1120 VALU at 65536);
// the packed pair halves the instructions per configuration but, at two configurations per
// lane, leaves half the SIMDs without a wave.  Here each pair of packed waves splits the work
// instead: the bias wave evaluates C = rnea(q, qd, 0) for 128 configurations (two per lane),
// the mass wave -- on another SIMD of the CU -- H and its L D L^T factorisation and, after one
// block barrier that hands it C through LDS, the solve: ~590 instructions per wave.  A
// 256-thread block covers one 256-configuration tile with two such pairs (waves 0/2 and 1/3:
// configurations [0,128) and [128,256)), so the grid keeps the one-per-lane kernel's wave
// count.  Both waves load q and evaluate (sin, cos); handing them over through LDS instead
// (one more barrier, q read once) measured slower: 4.38 vs 4.05 us at 65536 (HIP graph), the
// mass wave then waits for the bias wave's q rows.  Lanes past B read the tile's last
// configuration and store nothing; every wave reaches the barrier.
template <int N, bool FAST>
__device__ __forceinline__ void fdh_split_block2(const f2 *mdl, const float *__restrict__ q,
                                                 const float *__restrict__ qd, const float *__restrict__ tau,
                                                 float *__restrict__ qdd, uint32_t B, int64_t ld, int64_t bs) {
    __shared__ f2 shC[2][N][64];
    const uint32_t w = threadIdx.x >> 6, g = w & 1u, l = threadIdx.x & 63u;
    const uint32_t first = blockIdx.x * 256u;  // < B: the grid is ceil(B / 256) blocks
    const uint32_t cA = (g << 7) + l, cB = cA + 64u, last = B - 1u - first;
    const bool liveA = cA <= last, liveB = cB <= last;
    const uint32_t offA = (liveA ? cA : last) * 4u;
    const uint32_t offB = liveB ? cB * 4u : offA;
    const int64_t o = (int64_t)blockIdx.x * bs;
    if (w < 2) {
        f2 qv[N], qdv[N], cs[N], sn[N], C[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row2(q + o, j * ld, offA, offB);
            __builtin_amdgcn_sched_barrier(0);
            qdv[j] = ld_row2(qd + o, j * ld, offA, offB);
            __builtin_amdgcn_sched_barrier(0);
        }
        InputGuard<f2> gd;  // out-of-domain configurations: C, and so every qdd, NaN
        fdh_bias<f2, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
#pragma unroll
        for (int j = 0; j < N; ++j) shC[g][j][l] = gd.out(C[j]);
        __syncthreads();
    } else {
        f2 qv[N], tv[N], cs[N], sn[N], C[N], H[N][N], Di[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row2(q + o, j * ld, offA, offB);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            tv[j] = ld_row2(tau + o, j * ld, offA, offB);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) sin_cos<FAST>(qv[j], sn[j], cs[j]);
        fdh_factor<f2, N>(mdl, cs, sn, H, Di);
        // Everything above feeds only the liveA-guarded stores: without these pins the compiler
        // sinks the loads and the mass-matrix work past the barrier, and the mass wave would
        // start only after the bias wave has finished (5.69 vs 4.50 us at 65536, measured).
#pragma unroll
        for (int j = 0; j < N; ++j) {
            asm volatile("" : "+v"(Di[j].x), "+v"(Di[j].y));
            asm volatile("" : "+v"(tv[j].x), "+v"(tv[j].y));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; ++j) C[j] = shC[g][j][l];
        // a NaN in C (the bias wave's guard) reaches every qdd through the solve: every
        // y_i = tau_i - C_i is NaN, so is every forward and back substitution value
        InputGuard<f2> gd;
        gd.vals(tv);
        fdh_solve<f2, N>(H, Di, tv, C, [&](int j, f2 v) {
            if (liveA) st_row2(qdd + o, j * ld, offA, offB, gd.out(v));
        });
    }
}

// The same split one configuration per lane (jit pack 5; capi.cpp fd_pack takes it up to 2^17
// configurations, where it keeps every SIMD busy that the packed split would leave idle): a
// 256-thread block covers 128 configurations -- half a 256-configuration tile -- with two wave
// pairs (waves 0/2 and 1/3: configurations [0,64) and [64,128) of that half).  FR3 fp32 32768:
// 3.42 us vs 3.77 packed split, 4.08 one per lane (HIP graph).  fp64 measured slower at every
// size: its sincos is ~150 instructions, repeated by both waves.
template <typename T, int N, bool FAST>
__device__ __forceinline__ void fdh_split_block1(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                                 const T *__restrict__ tau, T *__restrict__ qdd, uint32_t B,
                                                 int64_t ld, int64_t bs) {
    __shared__ T shC[2][N][64];
    // The roles alternate by wave and block parity (w is a permutation of the wave index), so
    // the two blocks a CU holds put a bias wave and a mass-matrix wave on each SIMD rather than
    // two of one kind: FR3 fp32, HIP graph, 65536 4.15 vs 4.21 us, 131072 5.45 vs 5.53
    // (profiles/r06/mix/).
    const uint32_t wr = threadIdx.x >> 6;
    const uint32_t w = (((wr ^ blockIdx.x) & 1u) << 1) + (wr >> 1);
    const uint32_t g = w & 1u, l = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x >> 1, first = blockIdx.x * 128u;  // < B (grid ceil(B / 128))
    const uint32_t c = ((blockIdx.x & 1u) << 7) + (g << 6) + l;       // within the tile
    const uint32_t last = B - 1u - tile * 256u;
    const bool live = first + (g << 6) + l < B;
    const uint32_t off = (live ? c : last) * (uint32_t)sizeof(T);
    const int64_t o = (int64_t)tile * bs;
    if (w < 2) {
        T qv[N], qdv[N], cs[N], sn[N], C[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
            qdv[j] = ld_row(qd + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
        InputGuard<T> gd;  // as fdh_split_block2
        fdh_bias<T, N, FAST>(mdl, qv, qdv, cs, sn, C, gd);
#pragma unroll
        for (int j = 0; j < N; ++j) shC[g][j][l] = gd.out(C[j]);
        __syncthreads();
    } else {
        T qv[N], tv[N], cs[N], sn[N], C[N], H[N][N], Di[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            tv[j] = ld_row(tau + o, j * ld, off);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) sin_cos<FAST>(qv[j], sn[j], cs[j]);
        fdh_factor<T, N>(mdl, cs, sn, H, Di);
#pragma unroll
        for (int j = 0; j < N; ++j) {
            asm volatile("" : "+v"(Di[j]));
            asm volatile("" : "+v"(tv[j]));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < N; ++j) C[j] = shC[g][j][l];
        InputGuard<T> gd;
        gd.vals(tv);
        fdh_solve<T, N>(H, Di, tv, C, [&](int j, T v) {
            if (live) st_row(qdd + o, j * ld, off, gd.out(v));
        });
    }
}

}  // namespace dev
}  // namespace rbamd
