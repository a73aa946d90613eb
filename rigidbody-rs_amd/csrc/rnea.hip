// rnea.hip -- batched inverse dynamics (Multibody::rnea, multibody.rs:111-153).
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "rnea_body.hip.hpp"
#include "tuning.hpp"

namespace rbamd {
namespace dev {

// One configuration per lane; the grid covers the batch.  Block k's arrays start at
// element k * bstride: kBlock for SoA (x[j*ld + b]), N * kBlock for the tiled layout
// (ld = kBlock; kernels.hpp).
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void rnea_kernel(const T *__restrict__ gmdl,
                                                      const T *__restrict__ q,
                                                      const T *__restrict__ qd,
                                                      const T *__restrict__ qdd,
                                                      T *__restrict__ tau, uint32_t B,
                                                      int64_t ld, int64_t bstride) {
    __shared__ T mdl[N * kLinkStride];
    ModelStage<T, N, kBlock> st;
    st.fetch(gmdl);
    const int64_t o = (int64_t)blockIdx.x * bstride;
    q += o; qd += o; qdd += o; tau += o;
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t off = threadIdx.x * (uint32_t)sizeof(T);
    T qv[N], qdv[N], qddv[N];
    if (b < B) load_cfg<T, N>(q, qd, qdd, ld, off, qv, qdv, qddv);
    st.commit(mdl);
    if (b >= B) return;
    rnea_eval<T, N, FAST>(mdl, qv, qdv, qddv, [&](int j, T v) { st_row(tau, j * ld, off, v); });
}

// Streaming form (rnea_stream_lane): resident-sized grid, register prefetch.
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void rnea_stream_kernel(const T *__restrict__ gmdl,
                                                             const T *__restrict__ q,
                                                             const T *__restrict__ qd,
                                                             const T *__restrict__ qdd,
                                                             T *__restrict__ tau, uint32_t B,
                                                             int64_t ld) {
    __shared__ T mdl[N * kLinkStride];
    ModelStage<T, N, kBlock> st;
    st.fetch(gmdl);
    const uint32_t stride = gridDim.x * kBlock;
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    T qv[N], qdv[N], qddv[N];
    if (b < B) load_cfg<T, N>(q, qd, qdd, ld, b * (uint32_t)sizeof(T), qv, qdv, qddv);
    st.commit(mdl);
    if (b >= B) return;
    rnea_stream_lane<T, N, FAST>(mdl, q, qd, qdd, tau, b, stride, B, ld, qv, qdv, qddv);
}

}  // namespace dev

namespace {
template <typename T, int N, bool F>
hipError_t rnea_go(const T *mdl, const T *q, const T *qd, const T *qdd, T *tau, uint32_t B, int64_t ld,
                   hipStream_t s, bool tiled) {
    const Tuning &tn = tuning();
    const unsigned full = dev::grid_for(B);
    if (!tiled && rnea_use_stream(sizeof(T) == 8, N)) {
        auto kfn = dev::rnea_stream_kernel<T, N, F>;
        const unsigned g = stream_grid((const void *)kfn, dev::kBlock, full, tn.grid_factor);
        hipLaunchKernelGGL(kfn, dim3(g), dim3(dev::kBlock), 0, s, mdl, q, qd, qdd, tau, B, ld);
    } else {
        const int64_t bs = tiled ? (int64_t)N * dev::kBlock : dev::kBlock;
        hipLaunchKernelGGL((dev::rnea_kernel<T, N, F>), dim3(full), dim3(dev::kBlock), 0, s, mdl, q, qd, qdd, tau,
                           B, tiled ? (int64_t)dev::kBlock : ld, bs);
    }
    return hipGetLastError();
}
}  // namespace

template <typename T>
hipError_t launch_rnea(int n, const T *mdl, const T *q, const T *qd, const T *qdd, T *tau,
                       uint32_t B, int64_t ld, hipStream_t s, bool fast, bool tiled) {
    if (B == 0) return hipSuccess;
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        if constexpr (sizeof(T) == 4) {                                                          \
            if (fast) return rnea_go<T, N, true>(mdl, q, qd, qdd, tau, B, ld, s, tiled);                \
        }                                                                                        \
        return rnea_go<T, N, false>(mdl, q, qd, qdd, tau, B, ld, s, tiled);
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
}

template hipError_t launch_rnea<float>(int, const float *, const float *, const float *, const float *, float *, uint32_t, int64_t, hipStream_t, bool, bool);
template hipError_t launch_rnea<double>(int, const double *, const double *, const double *, const double *, double *, uint32_t, int64_t, hipStream_t, bool, bool);

}  // namespace rbamd
