// rnea_body.hip.hpp -- per-lane RNEA (device).  Shared by the precompiled kernels
// (rnea.hip, model constants staged in LDS) and the model-specialised kernels compiled
// at load time by hipRTC (jit.cpp, model constants as compile-time immediates).
#pragma once

#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

// ----------------------------------------------------------------------------- RNEA
// Per-link steps of the serial-chain RNEA, shared by the one-pass form (rnea_eval) and the
// segmented form (rnea_eval_seg) so both run the identical operation sequence.
template <typename T>
struct RneaState {
    V3<T> w, v, aw, av;  // link velocity / acceleration (rot, lin), link coordinates
};

// Link 0: v_{-1} = 0, a_{-1} = (0, (0,0,+g)) -- multibody.rs:116-120
template <typename T, bool FAST>
__device__ __forceinline__ void rnea_fwd0(const T *mdl, T q0, T qd0, T qdd0, RneaState<T> &st, T &sn, T &cs,
                                          V3<T> &fn, V3<T> &ff) {
    const Link<T> L = load_link(mdl, 0);
    sin_cos<FAST>(q0, sn, cs);
    const M3<T> E = joint_rotation(L.Rp, cs, sn);
    const T g = T(kGravity);
    st.w = v3(T(0), T(0), qd0);
    st.v = v3(T(0), T(0), T(0));
    st.aw = v3(T(0), T(0), qdd0);
    st.av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);  // E^T (0,0,g)
    // I v with v = (w, 0):  n = I_o w,  f = -h x w
    const V3<T> In = v3(L.Io.xz * qd0, L.Io.yz * qd0, L.Io.zz * qd0);
    const V3<T> If = v3(-L.h.y * qd0, L.h.x * qd0, T(0));  // -h x (0,0,qd)
    V3<T> An, Af;
    inertia_mul(L, st.aw, st.av, An, Af);
    ff = cross_add(Af, st.w, If);
    fn = cross_add(An, st.w, In);
}

// Link j >= 1: forward sweep step (multibody.rs:122-141).
template <typename T, bool FAST>
__device__ __forceinline__ void rnea_fwd(const T *mdl, int j, T qj, T qdj, T qddj, RneaState<T> &st, T &sn, T &cs,
                                         V3<T> &fn, V3<T> &ff) {
    const Link<T> L = load_link(mdl, j);
    sin_cos<FAST>(qj, sn, cs);
    const M3<T> E = joint_rotation(L.Rp, cs, sn);
    // SpatialVelocity::transform (spatial.rs:110-116) on v and a
    const V3<T> u = cross_sub(st.v, L.p, st.w);
    const V3<T> ua = cross_sub(st.av, L.p, st.aw);
    V3<T> wn = mul_t(E, st.w), vn = mul_t(E, u);
    V3<T> awn = mul_t(E, st.aw), avn = mul_t(E, ua);
    wn.z += qdj;        // multibody.rs:130
    awn.z += qddj;      // multibody.rs:133
    avn.x = fmadd(vn.y, qdj, avn.x);   // multibody.rs:135-138, v x (z qd) unrolled
    avn.y = fmadd(-vn.x, qdj, avn.y);
    awn.x = fmadd(wn.y, qdj, awn.x);
    awn.y = fmadd(-wn.x, qdj, awn.y);
    st.w = wn; st.v = vn; st.aw = awn; st.av = avn;
    // f = I a + v x* (I v)   (multibody.rs:140)
    V3<T> In, If, An, Af;
    inertia_mul(L, st.w, st.v, In, If);
    inertia_mul(L, st.aw, st.av, An, Af);
    ff = cross_add(Af, st.w, If);
    fn = cross_add(cross_add(An, st.w, In), st.v, If);
}

// Backward sweep step: f_{j-1} += X_j^-1 f_j  (multibody.rs:145-150).
template <typename T>
__device__ __forceinline__ void rnea_bwd(const T *mdl, int j, T cj, T sj, const V3<T> &ffj, const V3<T> &fnj,
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

// Forward sweep (multibody.rs:122-141) then backward sweep (143-150), fused: the
// per-link forces never leave registers.  One call evaluates the configuration whose
// joint values are in (qv, qdv, qddv) and hands tau_j to `out(j, value)`.
template <typename T, int N, bool FAST, typename Out>
__device__ __forceinline__ void rnea_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N],
                                          const T (&qddv)[N], Out &&out) {
    T cs[N], sn[N];
    V3<T> fn[N], ff[N];  // per-link spatial force: moment n (rot), force f (lin)
    RneaState<T> st;
    rnea_fwd0<T, FAST>(mdl, qv[0], qdv[0], qddv[0], st, sn[0], cs[0], fn[0], ff[0]);
#pragma unroll
    for (int j = 1; j < N; ++j) rnea_fwd<T, FAST>(mdl, j, qv[j], qdv[j], qddv[j], st, sn[j], cs[j], fn[j], ff[j]);

    // Backward sweep: tau_i = n_i.z (multibody.rs:144)
    reload_fence();
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        out(j, fn[j].z);
        rnea_bwd(mdl, j, cs[j], sn[j], ff[j], fn[j], ff[j - 1], fn[j - 1]);
    }
    out(0, fn[0].z);
}

// Segmented form for long chains: the per-link state the backward sweep needs (force 6,
// cos/sin 2 -- 8 values per link, 240 VGPRs for 30 links, 2 waves/SIMD) is held for one
// segment of ceil(N/S) links at a time.  Segments are processed top (leaf) first: each pass
// reloads the inputs of links 0..hi-1 (`load(j, q, qd, qdd)`; L2/MALL-resident after the
// first pass), recomputes the forward sweep up to its top link keeping only its own links'
// state, and runs its part of the backward sweep; the force of its lowest link is carried
// (with that link's cos/sin) into the next pass, where the same rnea_bwd step applies it --
// so every tau is computed by exactly the operations of rnea_eval (bit-identical), at
// (S+1)/2 times the forward-sweep work.
template <typename T, int N, int S, bool FAST, typename Load, typename Out>
__device__ __forceinline__ void rnea_eval_seg(const T *mdl, Load &&load, Out &&out) {
    constexpr int L = (N + S - 1) / S;
    T ccs = T(0), csn = T(0);
    V3<T> cff = v3(T(0), T(0), T(0)), cfn = cff;
    cfor_rev<S>([&](auto sc) {
        constexpr int seg = decltype(sc)::value;
        constexpr int lo = seg * L, hi = (lo + L < N) ? lo + L : N;
        if constexpr (lo < N) {
            T qv[hi], qdv[hi], qddv[hi];
            cfor<0, hi>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                load(j, qv[j], qdv[j], qddv[j]);
            });
            T cs[hi - lo], sn[hi - lo];
            V3<T> fn[hi - lo], ff[hi - lo];
            RneaState<T> st;
            cfor<0, hi>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                T s_, c_;
                V3<T> fn_, ff_;
                if constexpr (j == 0)
                    rnea_fwd0<T, FAST>(mdl, qv[0], qdv[0], qddv[0], st, s_, c_, fn_, ff_);
                else
                    rnea_fwd<T, FAST>(mdl, j, qv[j], qdv[j], qddv[j], st, s_, c_, fn_, ff_);
                if constexpr (j >= lo) {
                    sn[j - lo] = s_; cs[j - lo] = c_; fn[j - lo] = fn_; ff[j - lo] = ff_;
                }
            });
            reload_fence();
            if constexpr (hi < N) rnea_bwd(mdl, hi, ccs, csn, cff, cfn, ff[hi - 1 - lo], fn[hi - 1 - lo]);
            cfor_rev<hi - lo>([&](auto kc) {
                constexpr int k = decltype(kc)::value, j = lo + k;
                out(j, fn[k].z);
                if constexpr (k > 0) {
                    rnea_bwd(mdl, j, cs[k], sn[k], ff[k], fn[k], ff[k - 1], fn[k - 1]);
                } else if constexpr (j > 0) {
                    ccs = cs[0]; csn = sn[0]; cff = ff[0]; cfn = fn[0];
                }
            });
        }
    });
}

template <typename T, int N, bool FAST, typename Topo, typename Out>
__device__ __forceinline__ void rnea_any(const T *mdl, const T (&qv)[N], const T (&qdv)[N], const T (&qddv)[N],
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

// Segmented lane (model-specialised kernels of long serial chains, tuning rnea_seg): S
// segments, inputs reloaded per pass (rnea_eval_seg).
template <typename T, int N, int S, bool FAST>
__device__ __forceinline__ void rnea_lane_seg(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                              const T *__restrict__ qdd, T *__restrict__ tau, uint32_t b,
                                              int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    rnea_eval_seg<T, N, S, FAST>(
        mdl,
        [&](int j, T &x, T &y, T &z) {
            x = ld_row(q, j * ld, off);
            y = ld_row(qd, j * ld, off);
            z = ld_row(qdd, j * ld, off);
        },
        [&](int j, T v) { st_row(tau, j * ld, off, v); });
}

// Paired lane (fp32 model-specialised kernels, spatial.hip.hpp f2): the configurations at
// lane offset `off` of the batch blocks starting at elements oA and oB, evaluated together.
template <int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rnea_lane2(const f2 *mdl, const float *__restrict__ q, const float *__restrict__ qd,
                                           const float *__restrict__ qdd, float *__restrict__ tau, int64_t oA,
                                           int64_t oB, uint32_t off, int64_t ld) {
    f2 qv[N], qdv[N], qddv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row2(q, oA, oB, j * ld, off);
        qdv[j] = ld_row2(qd, oA, oB, j * ld, off);
        qddv[j] = ld_row2(qdd, oA, oB, j * ld, off);
    }
    rnea_any<f2, N, FAST, Topo>(mdl, qv, qdv, qddv, [&](int j, f2 v) { st_row2(tau, oA, oB, j * ld, off, v); });
}

// Streaming form: walk the batch with `stride`, prefetching the next configuration's
// joint values into registers before evaluating the current one.
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

// ------------------------------------------------------------------ LDS-tiled form
// A 256-thread block owns configurations [b0, b0+256).  Global traffic moves whole tile
// rows with 16-byte accesses (one 1 KiB wave-instruction per fp32 row; the probe in
// probe.hip measures 4-byte lanes at 3.8-3.9 TB/s vs 5.0-5.5 TB/s for 16-byte lanes on
// this pattern), and the per-lane math keeps one configuration per lane reading its
// values from LDS (conflict-free: lane t reads word t of a row).
template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
    using type = float4;
};
template <>
struct Vec16<double> {
    using type = double2;
};

constexpr int kTile = 256;

template <typename T, int ROWS>
__device__ __forceinline__ void tile_load(const T *__restrict__ a0, const T *__restrict__ a1,
                                          const T *__restrict__ a2, int rows_per_array, int64_t ld,
                                          uint32_t b0, T *tile) {
    using V = typename Vec16<T>::type;
    constexpr int VPL = 16 / (int)sizeof(T);  // values per 16-byte access
    constexpr int LPR = kTile / VPL;          // accesses per tile row
#pragma unroll
    for (int k0 = 0; k0 < ROWS * LPR; k0 += kTile) {
        const int k = k0 + (int)threadIdx.x;
        if (k < ROWS * LPR) {
            const int r = k / LPR, c = k % LPR;
            const int arr = r / rows_per_array, j = r % rows_per_array;
            const T *base = arr == 0 ? a0 : (arr == 1 ? a1 : a2);
            const V v = *reinterpret_cast<const V *>(base + j * ld + b0 + c * VPL);
            *reinterpret_cast<V *>(tile + r * kTile + c * VPL) = v;
        }
    }
}

template <typename T, int ROWS>
__device__ __forceinline__ void tile_store(T *__restrict__ dst, int64_t ld, uint32_t b0, const T *tile) {
    using V = typename Vec16<T>::type;
    constexpr int VPL = 16 / (int)sizeof(T);
    constexpr int LPR = kTile / VPL;
#pragma unroll
    for (int k0 = 0; k0 < ROWS * LPR; k0 += kTile) {
        const int k = k0 + (int)threadIdx.x;
        if (k < ROWS * LPR) {
            const int r = k / LPR, c = k % LPR;
            *reinterpret_cast<V *>(dst + r * ld + b0 + c * VPL) =
                *reinterpret_cast<const V *>(tile + r * kTile + c * VPL);
        }
    }
}

// Whole-block tile: caller guarantees b0 + 256 <= B and 16-byte alignment of every row
// start (base pointers and ld * sizeof(T) multiples of 16).  `tile` holds 3N rows.
template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void rnea_tile(const T *mdl, const T *__restrict__ q, const T *__restrict__ qd,
                                          const T *__restrict__ qdd, T *__restrict__ tau, uint32_t b0,
                                          int64_t ld, T *tile) {
    const int t = (int)threadIdx.x;
    tile_load<T, 3 * N>(q, qd, qdd, N, ld, b0, tile);
    __syncthreads();
    T qv[N], qdv[N], qddv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = tile[j * kTile + t];
        qdv[j] = tile[(N + j) * kTile + t];
        qddv[j] = tile[(2 * N + j) * kTile + t];
    }
    __syncthreads();  // every lane holds its inputs; rows 0..N-1 become the output tile
    rnea_any<T, N, FAST, Topo>(mdl, qv, qdv, qddv, [&](int j, T v) { tile[j * kTile + t] = v; });
    __syncthreads();
    tile_store<T, N>(tau, ld, b0, tile);
}

}  // namespace dev
}  // namespace rbamd
