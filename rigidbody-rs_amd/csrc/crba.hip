// crba.hip -- batched joint-space mass matrix (Multibody::crba, multibody.rs:155-174).
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "spatial.hip.hpp"
#include "artinertia.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------------------------------ CRBA
// multibody.rs:155-174: composite inertia leaf->root; column i of H from F = Ic_i S
// carried to the root.  Output matches the ABI: n x n column-major per configuration,
// H[j + n*i] for j <= i, strictly-lower entries written as exact zeros.
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void crba_kernel(const T *__restrict__ gmdl,
                                                      const T *__restrict__ q,
                                                      T *__restrict__ H, uint32_t B,
                                                      int64_t ld) {
    __shared__ T mdl[N * kLinkStride];
    stage_model<T, N, kBlock>(gmdl, mdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    const uint32_t off = b * (uint32_t)sizeof(T);
    T cs[N], sn[N];
#pragma unroll
    for (int j = 0; j < N; ++j) sin_cos<FAST>(ld_row(q, j * ld, off), sn[j], cs[j]);

    ArtI<T> Ic = rigid_inertia(load_link(mdl, N - 1));
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        reload_fence();
        st_row(H, (i + N * i) * ld, off, Ic.A.zz);  // get_rotz, inertia.rs:91-93
#pragma unroll
        for (int r = i + 1; r < N; ++r) st_row(H, (r + N * i) * ld, off, T(0));
        V3<T> Fn = v3(Ic.A.xz, Ic.A.yz, Ic.A.zz);
        V3<T> Ff = v3(Ic.B.m[6], Ic.B.m[7], Ic.B.m[8]);
#pragma unroll
        for (int j = i - 1; j >= 0; --j) {
            const Link<T> L = load_link(mdl, j + 1);
            const M3<T> E = joint_rotation(L.Rp, cs[j + 1], sn[j + 1]);
            const V3<T> fl = mul(E, Ff);
            Fn = cross_add(mul(E, Fn), L.p, fl);
            Ff = fl;
            st_row(H, (j + N * i) * ld, off, Fn.z);
        }
        if (i > 0) {
            const Link<T> L = load_link(mdl, i);
            const M3<T> E = joint_rotation(L.Rp, cs[i], sn[i]);
            Ic = to_parent(E, L.p, Ic);
            add_rigid(Ic, load_link(mdl, i - 1));
        }
    }
}

}  // namespace dev

template <typename T>
hipError_t launch_crba(int n, const T *mdl, const T *q, T *H, uint32_t B, int64_t ld,
                       hipStream_t s) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        hipLaunchKernelGGL((dev::crba_kernel<T, N, false>), grid, block, 0, s, mdl, q, H, B, ld); \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_crba<float>(int, const float *, const float *, float *, uint32_t, int64_t, hipStream_t);
template hipError_t launch_crba<double>(int, const double *, const double *, double *, uint32_t, int64_t, hipStream_t);

}  // namespace rbamd
