// batch_bench.cpp -- the batched C ABI (include/rigidbody_batch.h) as a native caller drives it:
// the loop a Rust / C++ MPC host would run, with no Python in it.  One device-resident batch of
// B configurations per call (FR3, B = 65536, fp32), inputs rotated
// over >= 1.25 GiB of device memory so the Infinity Cache cannot serve them, filled on device
// with the library's generator (the bench.py distributions: URDF joint limits, qdd +-10).
//
// Three timings of the same K calls (hipEvent pair on the launch stream, after warm-up):
//   eager   K back-to-back calls of the C entry point on one stream (host cost included when it
//           exceeds the device time: the launch-bound rate a caller gets without graphs)
//   host    the host time per call of that loop (std::chrono; the C ABI + hipModuleLaunchKernel),
//           beside the host time per launch of an empty kernel of the same grid (the runtime's
//           own floor)
//   graph   the same calls captured once into a HIP graph (100 per graph) and replayed
//
// usage: batch_bench KIND DTYPE B [K] [tiled]   KIND rnea|fd|rnea_fd|rnea+fd, DTYPE f32|f64
//   rnea_fd: multibody_rnea_fd_batch_* (tau = rnea(q, qd, qdd), qdd' = fd(q, qd, tau_in), one launch);
//   rnea+fd: the same pair as two calls, multibody_rnea_batch_* then multibody_fd_batch_* (config 4
//   before the fused entry point)
//   -> one JSON object on stdout.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rigidbody_batch.h"

// An empty kernel: the HIP runtime's own launch cost, against which the C ABI's host cost per
// call is read.
__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1024) *p = 0;
}

namespace {

#define CHECK_HIP(x)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

struct Set {
    void *in[4];  // q, qd, qdd | tau, tau_in (rnea_fd / rnea+fd)
    void *out[2];
};

enum Kind { kRnea, kFd, kRneaFd, kRneaThenFd };

template <typename T>
int call1(const Multibody *mb, bool fd, bool tiled, const T *a, const T *b, const T *c, T *o, int64_t B,
          hipStream_t st) {
    if constexpr (sizeof(T) == 4) {
        if (tiled) return fd ? multibody_fd_batch_tiled_f32(mb, a, b, c, o, B, st) : multibody_rnea_batch_tiled_f32(mb, a, b, c, o, B, st);
        return fd ? multibody_fd_batch_f32(mb, a, b, c, o, B, B, st) : multibody_rnea_batch_f32(mb, a, b, c, o, B, B, st);
    } else {
        if (tiled) return fd ? multibody_fd_batch_tiled_f64(mb, a, b, c, o, B, st) : multibody_rnea_batch_tiled_f64(mb, a, b, c, o, B, st);
        return fd ? multibody_fd_batch_f64(mb, a, b, c, o, B, B, st) : multibody_rnea_batch_f64(mb, a, b, c, o, B, B, st);
    }
}

template <typename T>
int call(const Multibody *mb, Kind kind, bool tiled, const Set &s, int64_t B, hipStream_t st) {
    const T *a = (const T *)s.in[0], *b = (const T *)s.in[1], *c = (const T *)s.in[2], *d = (const T *)s.in[3];
    T *o = (T *)s.out[0], *o2 = (T *)s.out[1];
    if (kind == kRnea || kind == kFd) return call1<T>(mb, kind == kFd, tiled, a, b, c, o, B, st);
    if (kind == kRneaThenFd) {
        if (int rc = call1<T>(mb, false, tiled, a, b, c, o, B, st)) return rc;
        return call1<T>(mb, true, tiled, a, b, d, o2, B, st);
    }
    if constexpr (sizeof(T) == 4) {
        return tiled ? multibody_rnea_fd_batch_tiled_f32(mb, a, b, c, d, o, o2, B, st)
                     : multibody_rnea_fd_batch_f32(mb, a, b, c, d, o, o2, B, B, st);
    } else {
        return tiled ? multibody_rnea_fd_batch_tiled_f64(mb, a, b, c, d, o, o2, B, st)
                     : multibody_rnea_fd_batch_f64(mb, a, b, c, d, o, o2, B, B, st);
    }
}

template <typename T>
int run(const char *kind_s, int64_t B, int K, bool tiled) {
    const Kind kind = !std::strcmp(kind_s, "fd") ? kFd : !std::strcmp(kind_s, "rnea_fd") ? kRneaFd
                      : !std::strcmp(kind_s, "rnea+fd") ? kRneaThenFd : kRnea;
    const bool fd = kind == kFd;
    const bool pair = kind == kRneaFd || kind == kRneaThenFd;
    const int nin = pair ? 4 : 3, nout = pair ? 2 : 1;
    // multibody_kernel_path_ex / _form_ex kind: 0 rnea, 1 fd, 6 rnea_fd
    const int qkind = kind == kFd ? 1 : kind == kRneaFd ? 6 : 0;
    Multibody *mb = multibody_new();
    if (!mb) {
        std::fprintf(stderr, "multibody_new: %s\n", rb_last_error());
        return 1;
    }
    const int n = multibody_dof(mb);
    std::vector<double> lo(n), hi(n), vel(n), eff(n);
    multibody_limits(mb, lo.data(), hi.data(), vel.data(), eff.data());
    // input ranges as chains.input_ranges: q in the limits, qd +-velocity, qdd +-10, tau +-effort
    std::vector<double> rlo[4], rhi[4];
    for (int k = 0; k < 4; ++k) rlo[k].resize(n), rhi[k].resize(n);
    for (int j = 0; j < n; ++j) {
        rlo[0][j] = std::isnan(lo[j]) ? -M_PI : lo[j];
        rhi[0][j] = std::isnan(hi[j]) ? M_PI : hi[j];
        rlo[1][j] = -vel[j], rhi[1][j] = vel[j];
        rlo[2][j] = fd ? -eff[j] : -10.0, rhi[2][j] = fd ? eff[j] : 10.0;
        rlo[3][j] = -eff[j], rhi[3][j] = eff[j];
    }
    // tiled arrays are [ceil(B/256)][n][256] (filled as SoA rows, then rb_to_tiled); SoA [n][B]
    const int64_t cols = tiled ? ((B + 255) / 256) * 256 : B;
    const size_t bytes = (size_t)n * (size_t)cols * sizeof(T);
    void *soa = nullptr;
    CHECK_HIP(hipMalloc(&soa, (size_t)n * (size_t)B * sizeof(T)));
    const int nsets = std::max<int>(2, (int)std::ceil(1.25 * (1 << 30) / ((nin + nout) * (double)bytes)));
    std::vector<Set> sets(nsets);
    hipStream_t st;
    CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int s = 0; s < nsets; ++s) {
        sets[s].in[3] = sets[s].out[1] = nullptr;
        for (int k = 0; k < nin; ++k) {
            CHECK_HIP(hipMalloc(&sets[s].in[k], bytes));
            void *dst = tiled ? soa : sets[s].in[k];
            int rc = sizeof(T) == 4 ? rb_fill_uniform_f32((float *)dst, n, B, B, rlo[k].data(), rhi[k].data(), 1000 * s + k, st)
                                    : rb_fill_uniform_f64((double *)dst, n, B, B, rlo[k].data(), rhi[k].data(), 1000 * s + k, st);
            if (!rc && tiled)
                rc = sizeof(T) == 4 ? rb_to_tiled_f32((const float *)soa, B, (float *)sets[s].in[k], n, B, st)
                                    : rb_to_tiled_f64((const double *)soa, B, (double *)sets[s].in[k], n, B, st);
            if (rc) {
                std::fprintf(stderr, "fill: %s\n", rb_last_error());
                return 1;
            }
        }
        for (int k = 0; k < nout; ++k) CHECK_HIP(hipMalloc(&sets[s].out[k], bytes));
    }
    CHECK_HIP(hipStreamSynchronize(st));
    CHECK_HIP(hipFree(soa));
    multibody_upload(mb);
    // pre-build the kernel this launch shape takes (hipRTC at first use), as INTEGRATION.md asks
    // before graph capture
    multibody_kernel_path_ex(mb, qkind, sizeof(T) == 8, B, tiled);
    if (kind == kRneaThenFd) multibody_kernel_path_ex(mb, 1, sizeof(T) == 8, B, tiled);
    auto launch = [&](int i) {
        if (call<T>(mb, kind, tiled, sets[i % nsets], B, st)) {
            std::fprintf(stderr, "launch: %s\n", rb_last_error());
            std::exit(1);
        }
    };
    for (int i = 0; i < 200; ++i) launch(i);
    CHECK_HIP(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    // eager
    CHECK_HIP(hipEventRecord(e0, st));
    auto h0 = std::chrono::steady_clock::now();
    for (int i = 0; i < K; ++i) launch(i);
    auto h1 = std::chrono::steady_clock::now();
    CHECK_HIP(hipEventRecord(e1, st));
    CHECK_HIP(hipEventSynchronize(e1));
    float eager_ms = 0;
    CHECK_HIP(hipEventElapsedTime(&eager_ms, e0, e1));
    const double host_us = std::chrono::duration<double, std::micro>(h1 - h0).count() / K;
    // the runtime's floor: K launches of an empty kernel of the same grid from this thread
    const unsigned grid = (unsigned)((B + 255) / 256);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, nullptr);
    CHECK_HIP(hipGetLastError());
    CHECK_HIP(hipStreamSynchronize(st));
    auto g0 = std::chrono::steady_clock::now();
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, st, nullptr);
    auto g1 = std::chrono::steady_clock::now();
    CHECK_HIP(hipStreamSynchronize(st));
    const double empty_host_us = std::chrono::duration<double, std::micro>(g1 - g0).count() / K;
    // graph: 100 consecutive calls captured once, replayed
    const int per = 100, reps = std::max(1, K / per);
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < per; ++i) launch(i);
    CHECK_HIP(hipStreamEndCapture(st, &g));
    CHECK_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 5; ++r) CHECK_HIP(hipGraphLaunch(ge, st));
    CHECK_HIP(hipStreamSynchronize(st));
    CHECK_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) CHECK_HIP(hipGraphLaunch(ge, st));
    CHECK_HIP(hipEventRecord(e1, st));
    CHECK_HIP(hipEventSynchronize(e1));
    float graph_ms = 0;
    CHECK_HIP(hipEventElapsedTime(&graph_ms, e0, e1));
    const double eager_us = eager_ms * 1e3 / K, graph_us = graph_ms * 1e3 / (reps * per);
    std::printf("{\"kind\": \"%s\", \"dtype\": \"%s\", \"batch\": %lld, \"layout\": \"%s\", \"calls\": %d, "
                "\"eager_us_per_call\": %.3f, \"host_us_per_call\": %.3f, \"empty_kernel_host_us\": %.3f, "
                "\"graph_us_per_call\": %.3f, "
                "\"eager_evals_per_s\": %.4g, \"graph_evals_per_s\": %.4g, \"input_sets\": %d, "
                "\"kernel_form\": %d}\n",
                kind_s, sizeof(T) == 4 ? "f32" : "f64", (long long)B, tiled ? "tiled" : "soa", K, eager_us, host_us,
                empty_host_us, graph_us, B / (eager_us * 1e-6), B / (graph_us * 1e-6), nsets,
                multibody_kernel_form_ex(mb, qkind, sizeof(T) == 8, B, tiled));
    CHECK_HIP(hipGraphExecDestroy(ge));
    CHECK_HIP(hipGraphDestroy(g));
    for (auto &s : sets) {
        for (void *p : s.in)
            if (p) CHECK_HIP(hipFree(p));
        for (void *p : s.out)
            if (p) CHECK_HIP(hipFree(p));
    }
    CHECK_HIP(hipStreamDestroy(st));
    multibody_free(mb);
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s rnea|fd|rnea_fd|rnea+fd f32|f64 B [K] [tiled]\n", argv[0]);
        return 2;
    }
    const int64_t B = std::atoll(argv[3]);
    const int K = argc > 4 ? std::max(100, std::atoi(argv[4])) : 20000;
    const bool tiled = argc > 5 && std::strcmp(argv[5], "tiled") == 0;
    if (B < 1) return 2;
    return std::strcmp(argv[2], "f64") == 0 ? run<double>(argv[1], B, K, tiled) : run<float>(argv[1], B, K, tiled);
}
