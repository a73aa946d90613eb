// rnea.hip -- batched inverse dynamics (Multibody::rnea, multibody.rs:111-153).
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "spatial.hip.hpp"

namespace rbamd {
namespace dev {

// ----------------------------------------------------------------------------- RNEA
// Forward sweep (multibody.rs:122-141) then backward sweep (143-150), fused: the
// per-link forces never leave registers.
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void rnea_kernel(const T *__restrict__ gmdl,
                                                      const T *__restrict__ q,
                                                      const T *__restrict__ qd,
                                                      const T *__restrict__ qdd,
                                                      T *__restrict__ tau, uint32_t B,
                                                      int64_t ld) {
    __shared__ T mdl[N * kLinkStride];
    stage_model<T, N, kBlock>(gmdl, mdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    const uint32_t off = b * (uint32_t)sizeof(T);

    T qv[N], qdv[N], qddv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        qv[j] = ld_row(q, j * ld, off);
        qdv[j] = ld_row(qd, j * ld, off);
        qddv[j] = ld_row(qdd, j * ld, off);
    }

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
        st_row(tau, j * ld, off, fn[j].z);
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
    st_row(tau, 0, off, fn[0].z);
}

}  // namespace dev

template <typename T>
hipError_t launch_rnea(int n, const T *mdl, const T *q, const T *qd, const T *qdd, T *tau,
                       uint32_t B, int64_t ld, hipStream_t s, bool fast) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        if constexpr (sizeof(T) == 4) {                                                          \
            if (fast)                                                                            \
                hipLaunchKernelGGL((dev::rnea_kernel<T, N, true>), grid, block, 0, s, mdl, q, qd, qdd, tau, B, ld); \
            else                                                                                 \
                hipLaunchKernelGGL((dev::rnea_kernel<T, N, false>), grid, block, 0, s, mdl, q, qd, qdd, tau, B, ld); \
        } else {                                                                                 \
            hipLaunchKernelGGL((dev::rnea_kernel<T, N, false>), grid, block, 0, s, mdl, q, qd, qdd, tau, B, ld); \
        }                                                                                        \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_rnea<float>(int, const float *, const float *, const float *, const float *, float *, uint32_t, int64_t, hipStream_t, bool);
template hipError_t launch_rnea<double>(int, const double *, const double *, const double *, const double *, double *, uint32_t, int64_t, hipStream_t, bool);

}  // namespace rbamd
