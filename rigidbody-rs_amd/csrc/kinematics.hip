// kinematics.hip -- batched fwd_kin / jac (multibody.rs:87-108) and synthetic input fill.
// Shared design notes: kernels.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"
#include "spatial.hip.hpp"

namespace rbamd {
namespace dev {

// ------------------------------------------------------------------- fwd_kin / jac
template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void fwd_kin_kernel(const T *__restrict__ gmdl,
                                                         const T *__restrict__ q,
                                                         T *__restrict__ pos, uint32_t B,
                                                         int64_t ld, int64_t bs_in, int64_t bs_out) {
    __shared__ T mdl[N * kLinkStride];
    stage_model<T, N, kBlock>(gmdl, mdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    q += (int64_t)blockIdx.x * bs_in;  // block k's rows (crba.hip)
    pos += (int64_t)blockIdx.x * bs_out;
    const uint32_t off = threadIdx.x * (uint32_t)sizeof(T);
    T qv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<SerialTopo>(qv);
    // T_0 T_1 ... T_{n-1} accumulated from the base: p += R p_i, R = R E_i
    M3<T> R{{T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1)}};
    V3<T> p = v3(T(0), T(0), T(0));
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const Link<T> L = load_link(mdl, j);
        T s, c;
        sin_cos<FAST>(qv[j], s, c);
        const M3<T> E = joint_rotation(L.Rp, c, s);
        p = mul_add(p, R, L.p);
        M3<T> Rn;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                Rn.m[3 * r + cc] = fmadd(R.m[3 * r + 0], E.m[cc], fmadd(R.m[3 * r + 1], E.m[3 + cc], R.m[3 * r + 2] * E.m[6 + cc]));
        R = Rn;
    }
    st_row(pos, 0 * ld, off, gd.out(p.x));
    st_row(pos, 1 * ld, off, gd.out(p.y));
    st_row(pos, 2 * ld, off, gd.out(p.z));
}

template <typename T, int N, bool FAST>
__global__ __launch_bounds__(kBlock) void jac_kernel(const T *__restrict__ gmdl,
                                                     const T *__restrict__ q,
                                                     T *__restrict__ J, uint32_t B,
                                                     int64_t ld, int64_t bs_in, int64_t bs_out) {
    __shared__ T mdl[N * kLinkStride];
    stage_model<T, N, kBlock>(gmdl, mdl);
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    q += (int64_t)blockIdx.x * bs_in;
    J += (int64_t)blockIdx.x * bs_out;
    const uint32_t off = threadIdx.x * (uint32_t)sizeof(T);
    // every angle first: a bad one poisons all columns, also those stored before it is used
    T qv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    InputGuard<T> gd;  // out-of-domain configurations: NaN outputs (spatial.hip.hpp)
    gd.template joints<SerialTopo>(qv);
    // acc = pose of the last frame in frame i, built leaf -> root (multibody.rs:97-106):
    // column i = motion transform of S_i = (0,0,1 | 0) by acc:
    //   rot = R^T z,  lin = R^T (0 - p x z) = -R^T (p.y, -p.x, 0)
    // Starts at the model tail (layout.hpp kTailOut): identity for z-axis chains, the last
    // link's axis-frame change otherwise, so columns come out in the URDF link frame.
    M3<T> R;
#pragma unroll
    for (int k = 0; k < 9; ++k) R.m[k] = gmdl[N * kLinkStride + k];
    V3<T> p = v3(T(0), T(0), T(0));
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        const V3<T> rot = v3(R.m[6], R.m[7], R.m[8]);
        const V3<T> lin = mul_t(R, v3(-p.y, p.x, T(0)));
        st_row(J, (6 * i + 0) * ld, off, gd.out(lin.x));
        st_row(J, (6 * i + 1) * ld, off, gd.out(lin.y));
        st_row(J, (6 * i + 2) * ld, off, gd.out(lin.z));
        st_row(J, (6 * i + 3) * ld, off, gd.out(rot.x));
        st_row(J, (6 * i + 4) * ld, off, gd.out(rot.y));
        st_row(J, (6 * i + 5) * ld, off, gd.out(rot.z));
        const Link<T> L = load_link(mdl, i);
        T s, c;
        sin_cos<FAST>(qv[i], s, c);
        const M3<T> E = joint_rotation(L.Rp, c, s);
        // acc <- T_i * acc = (E R, p_i + E p)
        p = mul_add(L.p, E, p);
        M3<T> Rn;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc)
                Rn.m[3 * r + cc] = fmadd(E.m[3 * r + 0], R.m[cc], fmadd(E.m[3 * r + 1], R.m[3 + cc], E.m[3 * r + 2] * R.m[6 + cc]));
        R = Rn;
    }
}

// ------------------------------------------------------------------ layout conversion
// One block per 256-configuration tile; both sides coalesced (a wave moves 64 consecutive
// elements of one row).
template <typename T>
__global__ __launch_bounds__(kBlock) void to_tiled_kernel(const T *__restrict__ src, int64_t ld,
                                                          T *__restrict__ dst, int rows, uint32_t B) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    T *t = dst + (int64_t)blockIdx.x * rows * kBlock + threadIdx.x;
    for (int r = 0; r < rows; ++r) t[(int64_t)r * kBlock] = b < B ? src[(int64_t)r * ld + b] : T(0);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void from_tiled_kernel(const T *__restrict__ src, T *__restrict__ dst,
                                                            int64_t ld, int rows, uint32_t B) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    const T *t = src + (int64_t)blockIdx.x * rows * kBlock + threadIdx.x;
    for (int r = 0; r < rows; ++r) dst[(int64_t)r * ld + b] = t[(int64_t)r * kBlock];
}

// ---------------------------------------------------------------- synthetic inputs
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(kBlock) void fill_uniform_kernel(T *__restrict__ x, int rows,
                                                              uint32_t B, int64_t ld,
                                                              const double *__restrict__ lohi,
                                                              uint64_t seed) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    const uint32_t off = b * (uint32_t)sizeof(T);
    for (int j = 0; j < rows; ++j) {
        const uint64_t idx = ((uint64_t)j << 40) | (uint64_t)b;
        const uint64_t u = splitmix64(seed * 0x9E3779B97F4A7C15ull + idx + 1ull);
        double r;
        if constexpr (sizeof(T) == 8) {
            r = (double)(u >> 11) * 0x1.0p-53;
        } else {
            r = (double)(u >> 40) * 0x1.0p-24;
        }
        const double lo = lohi[2 * j], hi = lohi[2 * j + 1];
        // no FMA contraction: the host reproduction (chains.host_uniform) rounds the
        // product and the sum separately
        {
#pragma clang fp contract(off)
            const double prod = (hi - lo) * r;
            st_row(x, j * ld, off, (T)(lo + prod));
        }
    }
}

}  // namespace dev

template <typename T>
hipError_t launch_fwd_kin(int n, const T *mdl, const T *q, T *pos, uint32_t B, int64_t ld,
                          hipStream_t s, bool fast, bool tiled) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    const int64_t lda = tiled ? dev::kBlock : ld, bs_in = tiled ? (int64_t)n * dev::kBlock : dev::kBlock,
                  bs_out = tiled ? 3 * dev::kBlock : dev::kBlock;
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        if (fast)                                                                               \
            hipLaunchKernelGGL((dev::fwd_kin_kernel<T, N, true>), grid, block, 0, s, mdl, q, pos, B, lda, bs_in, bs_out); \
        else                                                                                    \
            hipLaunchKernelGGL((dev::fwd_kin_kernel<T, N, false>), grid, block, 0, s, mdl, q, pos, B, lda, bs_in, bs_out); \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_jac(int n, const T *mdl, const T *q, T *J, uint32_t B, int64_t ld,
                      hipStream_t s, bool fast, bool tiled) {
    if (B == 0) return hipSuccess;
    const dim3 grid(dev::grid_for(B)), block(dev::kBlock);
    const int64_t lda = tiled ? dev::kBlock : ld, bs_in = tiled ? (int64_t)n * dev::kBlock : dev::kBlock,
                  bs_out = tiled ? 6 * (int64_t)n * dev::kBlock : dev::kBlock;
    switch (n) {
#define RB_CASE(N)                                                                              \
    case N:                                                                                     \
        if (fast)                                                                               \
            hipLaunchKernelGGL((dev::jac_kernel<T, N, true>), grid, block, 0, s, mdl, q, J, B, lda, bs_in, bs_out); \
        else                                                                                    \
            hipLaunchKernelGGL((dev::jac_kernel<T, N, false>), grid, block, 0, s, mdl, q, J, B, lda, bs_in, bs_out); \
        break;
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_fill_uniform(T *x, int rows, uint32_t B, int64_t ld, const double *lohi_dev,
                               uint64_t seed, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL((dev::fill_uniform_kernel<T>), dim3(dev::grid_for(B)), dim3(dev::kBlock), 0, s,
                       x, rows, B, ld, lohi_dev, seed);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_to_tiled(const T *src, int64_t ld, T *dst, int rows, uint32_t B, hipStream_t s) {
    if (B == 0 || rows == 0) return hipSuccess;
    hipLaunchKernelGGL((dev::to_tiled_kernel<T>), dim3(dev::grid_for(B)), dim3(dev::kBlock), 0, s, src, ld, dst,
                       rows, B);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_from_tiled(const T *src, T *dst, int64_t ld, int rows, uint32_t B, hipStream_t s) {
    if (B == 0 || rows == 0) return hipSuccess;
    hipLaunchKernelGGL((dev::from_tiled_kernel<T>), dim3(dev::grid_for(B)), dim3(dev::kBlock), 0, s, src, dst, ld,
                       rows, B);
    return hipGetLastError();
}

template hipError_t launch_to_tiled<float>(const float *, int64_t, float *, int, uint32_t, hipStream_t);
template hipError_t launch_to_tiled<double>(const double *, int64_t, double *, int, uint32_t, hipStream_t);
template hipError_t launch_from_tiled<float>(const float *, float *, int64_t, int, uint32_t, hipStream_t);
template hipError_t launch_from_tiled<double>(const double *, double *, int64_t, int, uint32_t, hipStream_t);
template hipError_t launch_fwd_kin<double>(int, const double *, const double *, double *, uint32_t, int64_t, hipStream_t,
                                           bool, bool);
template hipError_t launch_jac<double>(int, const double *, const double *, double *, uint32_t, int64_t, hipStream_t,
                                       bool, bool);
template hipError_t launch_fwd_kin<float>(int, const float *, const float *, float *, uint32_t, int64_t, hipStream_t,
                                          bool, bool);
template hipError_t launch_jac<float>(int, const float *, const float *, float *, uint32_t, int64_t, hipStream_t, bool, bool);
template hipError_t launch_fill_uniform<float>(float *, int, uint32_t, int64_t, const double *, uint64_t, hipStream_t);
template hipError_t launch_fill_uniform<double>(double *, int, uint32_t, int64_t, const double *, uint64_t, hipStream_t);

}  // namespace rbamd
