// rnea_body.hip.hpp -- per-lane RNEA (device).  Shared by the precompiled kernels
// (rnea.hip, model constants staged in LDS) and the model-specialised kernels compiled
// at load time by hipRTC (jit.cpp, model constants as compile-time immediates).
#pragma once

#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

// ----------------------------------------------------------------------------- RNEA
// Forward sweep (multibody.rs:122-141) then backward sweep (143-150), fused: the
// per-link forces never leave registers.  One call evaluates the configuration whose
// joint values are in (qv, qdv, qddv) and hands tau_j to `out(j, value)`.
template <typename T, int N, bool FAST, typename Out>
__device__ __forceinline__ void rnea_eval(const T *mdl, const T (&qv)[N], const T (&qdv)[N],
                                          const T (&qddv)[N], Out &&out) {
    T cs[N], sn[N];
    V3<T> fn[N], ff[N];  // per-link spatial force: moment n (rot), force f (lin)
    V3<T> w, v, aw, av;  // link velocity / acceleration (rot, lin), link coordinates

    {  // link 0: v_{-1} = 0, a_{-1} = (0, (0,0,+g)) -- multibody.rs:116-120
        const Link<T> L = load_link(mdl, 0);
        sin_cos<FAST>(qv[0], sn[0], cs[0]);
        const M3<T> E = joint_rotation(L.Rp, cs[0], sn[0]);
        const T g = T(kGravity);
        const T qd0 = qdv[0];
        w = v3(T(0), T(0), qd0);
        v = v3(T(0), T(0), T(0));
        aw = v3(T(0), T(0), qddv[0]);
        av = v3(g * E.m[6], g * E.m[7], g * E.m[8]);  // E^T (0,0,g)
        // I v with v = (w, 0):  n = I_o w,  f = -h x w
        const V3<T> In = v3(L.Io.xz * qd0, L.Io.yz * qd0, L.Io.zz * qd0);
        const V3<T> If = v3(-L.h.y * qd0, L.h.x * qd0, T(0));  // -h x (0,0,qd)
        V3<T> An, Af;
        inertia_mul(L, aw, av, An, Af);
        ff[0] = cross_add(Af, w, If);
        fn[0] = cross_add(An, w, In);
    }
#pragma unroll
    for (int j = 1; j < N; ++j) {
        const Link<T> L = load_link(mdl, j);
        sin_cos<FAST>(qv[j], sn[j], cs[j]);
        const M3<T> E = joint_rotation(L.Rp, cs[j], sn[j]);
        const T qdj = qdv[j];
        // SpatialVelocity::transform (spatial.rs:110-116) on v and a
        const V3<T> u = cross_sub(v, L.p, w);
        const V3<T> ua = cross_sub(av, L.p, aw);
        V3<T> wn = mul_t(E, w), vn = mul_t(E, u);
        V3<T> awn = mul_t(E, aw), avn = mul_t(E, ua);
        wn.z += qdj;        // multibody.rs:130
        awn.z += qddv[j];   // multibody.rs:133
        avn.x = fmadd(vn.y, qdj, avn.x);   // multibody.rs:135-138, v x (z qd) unrolled
        avn.y = fmadd(-vn.x, qdj, avn.y);
        awn.x = fmadd(wn.y, qdj, awn.x);
        awn.y = fmadd(-wn.x, qdj, awn.y);
        w = wn; v = vn; aw = awn; av = avn;
        // f = I a + v x* (I v)   (multibody.rs:140)
        V3<T> In, If, An, Af;
        inertia_mul(L, w, v, In, If);
        inertia_mul(L, aw, av, An, Af);
        ff[j] = cross_add(Af, w, If);
        fn[j] = cross_add(cross_add(An, w, In), v, If);
    }

    // Backward sweep: tau_i = n_i.z; f_{i-1} += X_i^-1 f_i  (multibody.rs:143-150)
    reload_fence();
#pragma unroll
    for (int j = N - 1; j >= 1; --j) {
        out(j, fn[j].z);
        const T *c = mdl + j * kLinkStride;
        const M3<T> Rp{{c[kE0 + 0], c[kE0 + 1], c[kE0 + 2], c[kE0 + 3], c[kE0 + 4], c[kE0 + 5],
                        c[kE0 + 6], c[kE0 + 7], c[kE0 + 8]}};
        const V3<T> p = v3(c[kP + 0], c[kP + 1], c[kP + 2]);
        const T cj = cs[j], sj = sn[j];
        // E x = R_p (Rz x)
        const V3<T> zf = v3(fmadd(cj, ff[j].x, -sj * ff[j].y), fmadd(sj, ff[j].x, cj * ff[j].y), ff[j].z);
        const V3<T> zn = v3(fmadd(cj, fn[j].x, -sj * fn[j].y), fmadd(sj, fn[j].x, cj * fn[j].y), fn[j].z);
        const V3<T> fl = mul(Rp, zf);
        ff[j - 1] = v3(ff[j - 1].x + fl.x, ff[j - 1].y + fl.y, ff[j - 1].z + fl.z);
        fn[j - 1] = cross_add(mul_add(fn[j - 1], Rp, zn), p, fl);
    }
    out(0, fn[0].z);
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
