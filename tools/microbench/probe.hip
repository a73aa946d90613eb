// probe.hip -- bandwidth probe with the RNEA access pattern (rows_in SoA rows read,
// rows_out rows written, no dynamics).  It measures the HBM ceiling the batched kernels
// can reach with a given per-lane access width: 4 B (one fp32 configuration per lane, what
// the kernels do), 8 B or 16 B (two / four consecutive configurations per lane).  Also used to calibrate
// rocprofv3 FETCH_SIZE / WRITE_SIZE against a known byte count.
//
// Measurement tooling, not product: built on its own as tools/microbench/libprobe.so
// (`make -C tools/microbench`), loaded by tools/probe_lib.py.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rbamd {
namespace dev {

constexpr int kBlock = 256;
inline unsigned grid_for(uint32_t n) { return (n + kBlock - 1) / kBlock; }

template <int W>
struct VecOf;
template <>
struct VecOf<1> {
    using type = float;
};
template <>
struct VecOf<2> {
    using type = float __attribute__((ext_vector_type(2)));
};
template <>
struct VecOf<4> {
    using type = float __attribute__((ext_vector_type(4)));
};

// All RI loads of a lane are issued before any use (compile-time row counts), as in the
// unrolled dynamics kernels.  NT bit 2 (value 4): tiled layout instead of SoA rows --
// element (row r, config b) at ((b / 256) * R + r) * 256 + b % 256, so one 256-config tile
// of all R rows is contiguous (ld unused).
template <int W, int RI, int RO, int NT>
__global__ __launch_bounds__(kBlock) void probe_rows_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                           uint32_t B, int64_t ld) {
    using V = typename VecOf<W>::type;
    const uint32_t b = (blockIdx.x * kBlock + threadIdx.x) * W;
    if (b >= B) return;
    constexpr bool kTiled = (NT & 4) != 0;
    const int64_t tile = (int64_t)(b >> 8), lane = b & 255u;
    V x[RI];
#pragma unroll
    for (int r = 0; r < RI; ++r) {
        const float *a = kTiled ? in + (tile * RI + r) * 256 + lane : in + r * ld + b;
        const V *p = reinterpret_cast<const V *>(a);
        x[r] = (NT & 1) ? __builtin_nontemporal_load(p) : *p;
    }
    V acc = x[0];
#pragma unroll
    for (int r = 1; r < RI; ++r) acc = acc + x[r];
#pragma unroll
    for (int r = 0; r < RO; ++r) {
        float *a = kTiled ? out + (tile * RO + r) * 256 + lane : out + r * ld + b;
        V *p = reinterpret_cast<V *>(a);
        if (NT & 2)
            __builtin_nontemporal_store(acc, p);
        else
            *p = acc;
    }
}

}  // namespace dev

namespace {
template <int RI, int RO, int NT>
hipError_t probe_go(const float *in, float *out, uint32_t B, int64_t ld, int width, hipStream_t s) {
    if (width == 4) {
        hipLaunchKernelGGL((dev::probe_rows_kernel<4, RI, RO, NT>), dim3(dev::grid_for(B / 4)), dim3(dev::kBlock), 0,
                           s, in, out, B, ld);
    } else if (width == 2) {
        hipLaunchKernelGGL((dev::probe_rows_kernel<2, RI, RO, NT>), dim3(dev::grid_for(B / 2)), dim3(dev::kBlock), 0,
                           s, in, out, B, ld);
    } else {
        hipLaunchKernelGGL((dev::probe_rows_kernel<1, RI, RO, NT>), dim3(dev::grid_for(B)), dim3(dev::kBlock), 0, s,
                           in, out, B, ld);
    }
    return hipGetLastError();
}

template <int RI, int RO>
hipError_t probe_nt(const float *in, float *out, uint32_t B, int64_t ld, int width, int nt, hipStream_t s) {
    switch (nt) {
        case 1: return probe_go<RI, RO, 1>(in, out, B, ld, width, s);
        case 2: return probe_go<RI, RO, 2>(in, out, B, ld, width, s);
        case 3: return probe_go<RI, RO, 3>(in, out, B, ld, width, s);
        case 4: return probe_go<RI, RO, 4>(in, out, B, ld, width, s);
        case 5: return probe_go<RI, RO, 5>(in, out, B, ld, width, s);
        case 6: return probe_go<RI, RO, 6>(in, out, B, ld, width, s);
        case 7: return probe_go<RI, RO, 7>(in, out, B, ld, width, s);
        default: return probe_go<RI, RO, 0>(in, out, B, ld, width, s);
    }
}
}  // namespace

// Row shapes of the dynamics kernels: 7-DOF (21 in / 7 out), 12-DOF, 30-DOF, 4/4, and the q-only kernels.
hipError_t launch_probe_rows(const float *in, float *out, int rows_in, int rows_out, uint32_t B, int64_t ld,
                             int width, hipStream_t s) {
    if (B == 0) return hipSuccess;
    // width encodes the non-temporal flags above the access width: width = w + 16*nt
    const int nt = width >> 4;
    width &= 15;
    if (B % width != 0 || ld % width != 0) return hipErrorInvalidValue;
    if ((nt & 4) && B % 256 != 0) return hipErrorInvalidValue;  // whole tiles only
    if (rows_in == 21 && rows_out == 7) return probe_nt<21, 7>(in, out, B, ld, width, nt, s);
    if (rows_in == 36 && rows_out == 12) return probe_nt<36, 12>(in, out, B, ld, width, nt, s);
    if (rows_in == 90 && rows_out == 30) return probe_nt<90, 30>(in, out, B, ld, width, nt, s);
    if (rows_in == 4 && rows_out == 4) return probe_nt<4, 4>(in, out, B, ld, width, nt, s);
    // the q-only kernels of FR3: CRBA (7 in / 49 out), Jacobian (7 / 42), forward
    // kinematics (7 / 3)
    if (rows_in == 7 && rows_out == 49) return probe_nt<7, 49>(in, out, B, ld, width, nt, s);
    if (rows_in == 7 && rows_out == 42) return probe_nt<7, 42>(in, out, B, ld, width, nt, s);
    if (rows_in == 7 && rows_out == 3) return probe_nt<7, 3>(in, out, B, ld, width, nt, s);
    return hipErrorInvalidValue;
}

}  // namespace rbamd

// Reads rows_in rows and writes rows_out rows of `batch` floats (width 1/2/4: 4/8/16 B per
// lane; + 16 * nt with nt bit 0 = non-temporal loads, bit 1 = non-temporal stores, bit 2 =
// tiled layout: element (row r, config b) at ((b / 256) * rows + r) * 256 + b % 256, batch a
// multiple of 256).  Returns a hipError_t code (0 = success).
extern "C" int rb_probe_rows_f32(const float *in, float *out, int rows_in, int rows_out, int64_t batch, int64_t ld,
                                 int width, void *stream) {
    if (!in || !out || rows_in < 1 || rows_out < 0 || batch < 0 || ld < batch || batch >= (int64_t(1) << 28))
        return (int)hipErrorInvalidValue;
    const int w = width & 15;
    if ((w != 1 && w != 2 && w != 4) || (width >> 4) > 7) return (int)hipErrorInvalidValue;
    return (int)rbamd::launch_probe_rows(in, out, rows_in, rows_out, (uint32_t)batch, ld, width, (hipStream_t)stream);
}
