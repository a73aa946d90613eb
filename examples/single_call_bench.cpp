// single_call_bench.cpp -- latency of the reference's single-configuration C ABI
// (rigidbody_bindings/rigidbody.h:11-16, lib.rs:15-70) as a C++ consumer sees it:
// the calls rigidbody_bindings/main.cpp:69-96 times with std::chrono, on the
// main.cpp:103-105 input, through librigidbody_bindings.so.  SURVEY §8(d) config 1.
//
// usage: single_call_bench [iters]   -> one JSON object on stdout:
//   {"iters": N, "rnea": {"median_us": .., "mean_us": .., "p99_us": .., "min_us": ..}, "crba": .., ...}
// Every returned buffer is freed with multibody_result_free (the reference leaks them).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rigidbody.h"

extern "C" void multibody_result_free(double *p);
extern "C" const char *rb_last_error(void);

namespace {

struct Stats {
    double median, mean, p99, min;
};

template <typename F>
bool measure(int iters, F &&call, Stats *out) {
    std::vector<double> us(iters);
    for (int i = 0; i < 50; ++i) {  // warm: model upload, kernel load, staging buffers
        double *r = call();
        if (!r) return false;
        multibody_result_free(r);
    }
    for (int i = 0; i < iters; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        double *r = call();
        auto t1 = std::chrono::steady_clock::now();
        if (!r) return false;
        multibody_result_free(r);
        us[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    double sum = 0;
    for (double u : us) sum += u;
    std::sort(us.begin(), us.end());
    out->median = us[iters / 2];
    out->mean = sum / iters;
    out->p99 = us[std::min(iters - 1, (iters * 99) / 100)];
    out->min = us[0];
    return true;
}

void print(const char *name, const Stats &s, bool last) {
    std::printf("\"%s\": {\"median_us\": %.3f, \"mean_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}%s", name,
                s.median, s.mean, s.p99, s.min, last ? "" : ", ");
}

}  // namespace

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::max(10, std::atoi(argv[1])) : 2000;
    double q[7] = {0.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0};    // main.cpp:103
    double dq[7] = {0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0};   // main.cpp:104
    double ddq[7] = {1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0};  // main.cpp:105
    Multibody *mb = multibody_new();
    if (!mb) {
        std::fprintf(stderr, "multibody_new failed: %s\n", rb_last_error());
        return 1;
    }
    Stats rnea, crba, jac, fk;
    bool ok = measure(iters, [&] { return multibody_rnea(mb, q, dq, ddq); }, &rnea) &&
              measure(iters, [&] { return multibody_crba(mb, q); }, &crba) &&
              measure(iters, [&] { return multibody_jac(mb, q); }, &jac) &&
              measure(iters, [&] { return multibody_fwd_kin(mb, q); }, &fk);
    if (!ok) {
        std::fprintf(stderr, "query failed: %s\n", rb_last_error());
        multibody_free(mb);
        return 1;
    }
    std::printf("{\"iters\": %d, ", iters);
    print("rnea", rnea, false);
    print("crba", crba, false);
    print("jac", jac, false);
    print("fwd_kin", fk, true);
    std::printf("}\n");
    multibody_free(mb);
    return 0;
}
