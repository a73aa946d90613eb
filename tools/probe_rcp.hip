// probe_rcp.hip -- relative error of the fp64 hardware reciprocal (v_rcp_f64) and of one / two
// Newton steps on it, over positive normal inputs spread across 2^-60 .. 2^60 (the pivots of
// the mass-matrix factorisation, spatial.hip.hpp recip).  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_rcp tools/probe_rcp.hip && tools/probe_rcp
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void rcp_kernel(const double *x, double *r0, double *r1, double *r2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    const double a = __builtin_amdgcn_rcp(v);
    const double b = __builtin_fma(a, __builtin_fma(-v, a, 1.0), a);
    const double c = __builtin_fma(b, __builtin_fma(-v, b, 1.0), b);
    r0[i] = a;
    r1[i] = b;
    r2[i] = c;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) * 0x1.0p-53;               // [0, 1)
        x[i] = std::ldexp(1.0 + u, (int)((s & 0x7f) % 121) - 60);      // [2^-60, 2^61)
    }
    double *dx, *d0, *d1, *d2;
    if (hipMalloc(&dx, n * 8) || hipMalloc(&d0, n * 8) || hipMalloc(&d1, n * 8) || hipMalloc(&d2, n * 8)) return 2;
    if (hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice)) return 3;
    rcp_kernel<<<(n + 255) / 256, 256>>>(dx, d0, d1, d2, n);
    if (hipGetLastError() || hipDeviceSynchronize()) return 4;
    std::vector<double> r0(n), r1(n), r2(n);
    if (hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost) || hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost) ||
        hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost))
        return 5;
    double e0 = 0, e1 = 0, e2 = 0;
    long exact1 = 0, exact2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double t = 1.0L / (long double)x[i];
        e0 = std::fmax(e0, (double)std::fabs((r0[i] - t) / t));
        e1 = std::fmax(e1, (double)std::fabs((r1[i] - t) / t));
        e2 = std::fmax(e2, (double)std::fabs((r2[i] - t) / t));
        exact1 += r1[i] == 1.0 / x[i];
        exact2 += r2[i] == 1.0 / x[i];
    }
    std::printf("{\"n\": %d, \"rcp_max_rel\": %.3e, \"newton1_max_rel\": %.3e, \"newton2_max_rel\": %.3e, "
                "\"newton1_correctly_rounded\": %.6f, \"newton2_correctly_rounded\": %.6f}\n",
                n, e0, e1, e2, (double)exact1 / n, (double)exact2 / n);
    (void)hipFree(dx); (void)hipFree(d0); (void)hipFree(d1); (void)hipFree(d2);
    return 0;
}
