// aba.hip -- batched forward dynamics by the Articulated-Body Algorithm.
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "aba_body.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------------------------------- ABA
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void aba_kernel(const T *__restrict__ gmdl,
                                                     const T *__restrict__ q,
                                                     const T *__restrict__ qd,
                                                     const T *__restrict__ tau,
                                                     T *__restrict__ qdd, uint32_t B,
                                                     int64_t ld, int64_t bstride) {
    __shared__ T mdl[N * kLinkStride];
    ModelStage<T, N, kBlock> st;
    st.fetch(gmdl);
    const int64_t o = (int64_t)blockIdx.x * bstride;  // SoA or tiled, as rnea_kernel
    q += o; qd += o; tau += o; qdd += o;
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t off = threadIdx.x * (uint32_t)sizeof(T);
    T qv[N], qdv[N], tv[N];
    if (b < B) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            qv[j] = ld_row(q, j * ld, off);
            qdv[j] = ld_row(qd, j * ld, off);
            tv[j] = ld_row(tau, j * ld, off);
        }
    }
    st.commit(mdl);
    if (b >= B) return;
    aba_eval<T, N, FAST>(mdl, qv, qdv, tv, [&](int j, T v) { st_row(qdd, j * ld, off, v); });
}

template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void rollout_kernel(const T *__restrict__ gmdl, T *__restrict__ q,
                                                         T *__restrict__ qd, const T *__restrict__ tau_seq, T dt,
                                                         int K, T *__restrict__ traj, uint32_t B, int64_t ld) {
    static_assert(kBlock == kRolloutBlock, "rollout LDS state is strided by the block size");
    __shared__ T mdl[N * kLinkStride];
    __shared__ RolloutShared<T, N> sh;
    ModelStage<T, N, kBlock> st;
    st.fetch(gmdl);
    st.commit(mdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    rollout_lane<T, N, FAST>(mdl, q, qd, tau_seq, dt, K, traj, b, ld, sh);
}

}  // namespace dev

template <typename T>
hipError_t launch_aba(int n, const T *mdl, const T *q, const T *qd, const T *tau, T *qdd,
                      uint32_t B, int64_t ld, hipStream_t s, bool fast, bool tiled) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    const int64_t lda = tiled ? (int64_t)dev::kBlock : ld;
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N: {                                                                                   \
        const int64_t bs = tiled ? (int64_t)N * dev::kBlock : dev::kBlock;                       \
        if (sizeof(T) == 4 && fast)                                                              \
            hipLaunchKernelGGL((dev::aba_kernel<T, N, sizeof(T) == 4>), grid, block, 0, s, mdl, q, qd, tau, qdd, B, \
                               lda, bs);                                                         \
        else                                                                                     \
            hipLaunchKernelGGL((dev::aba_kernel<T, N, false>), grid, block, 0, s, mdl, q, qd, tau, qdd, B, lda, bs); \
        break;                                                                                   \
    }
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_rollout(int n, const T *mdl, T *q, T *qd, const T *tau_seq, T dt, int K, T *traj, uint32_t B,
                          int64_t ld, hipStream_t s, bool fast) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    switch (n) {
#define RB_CASE(N)                                                                                        \
    case N:                                                                                               \
        if constexpr (sizeof(T) == 4) {                                                                    \
            if (fast) {                                                                                    \
                hipLaunchKernelGGL((dev::rollout_kernel<T, N, true>), grid, block, 0, s, mdl, q, qd, tau_seq, \
                                   dt, K, traj, B, ld);                                                    \
                break;                                                                                     \
            }                                                                                              \
        }                                                                                                  \
        hipLaunchKernelGGL((dev::rollout_kernel<T, N, false>), grid, block, 0, s, mdl, q, qd, tau_seq, dt, K,  \
                           traj, B, ld);                                                                   \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_rollout<float>(int, const float *, float *, float *, const float *, float, int, float *,
                                          uint32_t, int64_t, hipStream_t, bool);
template hipError_t launch_rollout<double>(int, const double *, double *, double *, const double *, double, int,
                                           double *, uint32_t, int64_t, hipStream_t, bool);
template hipError_t launch_aba<float>(int, const float *, const float *, const float *, const float *, float *, uint32_t, int64_t, hipStream_t, bool, bool);
template hipError_t launch_aba<double>(int, const double *, const double *, const double *, const double *, double *, uint32_t, int64_t, hipStream_t, bool, bool);

}  // namespace rbamd
