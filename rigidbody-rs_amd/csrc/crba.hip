// crba.hip -- batched joint-space mass matrix (Multibody::crba, multibody.rs:155-174).
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "crba_body.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------------------------------ CRBA
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void crba_kernel(const T *__restrict__ gmdl,
                                                      const T *__restrict__ q,
                                                      T *__restrict__ H, uint32_t B,
                                                      int64_t ld, int64_t bs_in, int64_t bs_out) {
    __shared__ T mdl[N * kLinkStride];
    ModelStage<T, N, kBlock> st;
    st.fetch(gmdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    // block k's rows start at element k * bs (SoA: 256, ld the row stride; tiled: rows * 256, ld 256)
    q += (int64_t)blockIdx.x * bs_in;
    H += (int64_t)blockIdx.x * bs_out;
    const uint32_t off = threadIdx.x * (uint32_t)sizeof(T);
    T qv[N];
    if (b < B) {
#pragma unroll
        for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    }
    st.commit(mdl);
    if (b >= B) return;
    crba_eval<T, N, FAST>(mdl, qv, [&](int e, T v) { st_row(H, e * ld, off, v); });
}

}  // namespace dev

template <typename T>
hipError_t launch_crba(int n, const T *mdl, const T *q, T *H, uint32_t B, int64_t ld,
                       hipStream_t s, bool tiled) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    const int64_t lda = tiled ? dev::kBlock : ld, bs_in = tiled ? (int64_t)n * dev::kBlock : dev::kBlock,
                  bs_out = tiled ? (int64_t)n * n * dev::kBlock : dev::kBlock;
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        hipLaunchKernelGGL((dev::crba_kernel<T, N, false>), grid, block, 0, s, mdl, q, H, B, lda, bs_in, bs_out); \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template hipError_t launch_crba<float>(int, const float *, const float *, float *, uint32_t, int64_t, hipStream_t, bool);
template hipError_t launch_crba<double>(int, const double *, const double *, double *, uint32_t, int64_t, hipStream_t,
                                        bool);

}  // namespace rbamd
