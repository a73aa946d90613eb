// probe.hip -- bandwidth probe with the RNEA access pattern (rows_in SoA rows read,
// rows_out rows written, no dynamics).  It measures the HBM ceiling the batched kernels
// can reach with a given per-lane access width: 4 B (one configuration per lane, what the
// kernels do) or 16 B (four consecutive configurations per lane).  Also used to calibrate
// rocprofv3 FETCH_SIZE / WRITE_SIZE against a known byte count.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dofs.hpp"
#include "kernels.hpp"

namespace rbamd {
namespace dev {

template <int W>
struct VecOf;
template <>
struct VecOf<1> {
    using type = float;
};
template <>
struct VecOf<4> {
    using type = float4;
};

template <int W>
__global__ __launch_bounds__(kBlock) void probe_rows_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                           int rows_in, int rows_out, uint32_t B, int64_t ld) {
    using V = typename VecOf<W>::type;
    const uint32_t b = (blockIdx.x * kBlock + threadIdx.x) * W;
    if (b >= B) return;
    V acc{};
    for (int r = 0; r < rows_in; ++r) acc = acc + *reinterpret_cast<const V *>(in + r * ld + b);
    for (int r = 0; r < rows_out; ++r) *reinterpret_cast<V *>(out + r * ld + b) = acc;
}

}  // namespace dev

hipError_t launch_probe_rows(const float *in, float *out, int rows_in, int rows_out, uint32_t B, int64_t ld,
                             int width, hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (width == 4) {
        if (B % 4 != 0 || ld % 4 != 0) return hipErrorInvalidValue;
        hipLaunchKernelGGL(dev::probe_rows_kernel<4>, dim3(dev::grid_for(B / 4)), dim3(dev::kBlock), 0, s, in, out,
                           rows_in, rows_out, B, ld);
    } else {
        hipLaunchKernelGGL(dev::probe_rows_kernel<1>, dim3(dev::grid_for(B)), dim3(dev::kBlock), 0, s, in, out,
                           rows_in, rows_out, B, ld);
    }
    return hipGetLastError();
}

}  // namespace rbamd
