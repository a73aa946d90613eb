// valu_issue.hip -- one-wave-per-SIMD VALU issue cost on gfx950, to decide the small-batch
// kernel forms: cycles per instruction for v_fma_f32 vs v_pk_fma_f32, with
// independent (8 chains) and dependent (1 chain) operands, all 64 lanes active vs only
// lanes 0..31 (the upper half of EXEC zero).  s_memtime around the loop, one wave per
// SIMD (grid = 4 x CUs blocks of 64 threads).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

template <int MODE, int CHAINS>
__global__ __launch_bounds__(64) void chain_kernel(float *out, long long *cyc, int half, float seed) {
    if (half && threadIdx.x >= 32) return;
    float a[CHAINS];
    f2 b[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
        a[k] = seed + threadIdx.x + k;
        b[k] = f2{a[k], a[k] + 1.f};
    }
    const float m = 0.999f + seed * 1e-9f;
    const f2 m2 = f2{m, m};
    const f2 c2 = f2{1e-3f, 2e-3f};
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) {
            if constexpr (MODE == 0) a[k] = __builtin_fmaf(a[k], m, 1e-3f);
            else b[k] = __builtin_elementwise_fma(b[k], m2, c2);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) s += (MODE == 0) ? a[k] : b[k].x + b[k].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int CHAINS>
void run(const char *name, int grid, float *dout, long long *dcyc, int half, int waves_per_simd = 1) {
    hipLaunchKernelGGL((chain_kernel<MODE, CHAINS>), dim3(grid), dim3(64), 0, 0, dout, dcyc, half, 1.0f);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((chain_kernel<MODE, CHAINS>), dim3(grid), dim3(64), 0, 0, dout, dcyc, half, 1.0f);
    hipDeviceSynchronize();
    std::vector<long long> c(grid);
    hipMemcpy(c.data(), dcyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
    double sum = 0;
    for (auto x : c) sum += (double)x;
    const double per = sum / grid / ((double)kIters * CHAINS);
    printf("{\"op\": \"%s\", \"chains\": %d, \"half_exec\": %d, \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.3f, \"simd_cycles_per_instr\": %.3f}\n",
           name, CHAINS, half, waves_per_simd, per, per / waves_per_simd);
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = 4 * cus;
    float *dout;
    long long *dcyc;
    hipMalloc(&dout, 8 * grid * 64 * sizeof(float));
    hipMalloc(&dcyc, 8 * grid * sizeof(long long));
    // several waves per SIMD: the grid holds k waves per SIMD, all resident at once (tiny kernels)
    for (int k : {2, 4, 8}) {
        run<0, 8>("v_fma_f32", k * grid, dout, dcyc, 0, k);
        run<1, 8>("v_pk_fma_f32", k * grid, dout, dcyc, 0, k);
        run<0, 1>("v_fma_f32", k * grid, dout, dcyc, 0, k);
        run<1, 1>("v_pk_fma_f32", k * grid, dout, dcyc, 0, k);
    }
    for (int half = 0; half < 2; ++half) {
        run<0, 1>("v_fma_f32", grid, dout, dcyc, half);
        run<0, 8>("v_fma_f32", grid, dout, dcyc, half);
        run<1, 1>("v_pk_fma_f32", grid, dout, dcyc, half);
        run<1, 8>("v_pk_fma_f32", grid, dout, dcyc, half);
    }
    return 0;
}
