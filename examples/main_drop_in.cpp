// main_drop_in.cpp -- the rigidbody half of the reference consumer
// (rigidbody_bindings/main.cpp:66-98, 101-115) built against this repo's
// include/rigidbody.h and librigidbody_bindings.so, unchanged in its use of the ABI:
// multibody_new / _rnea / _jac / _fwd_kin / _crba / _free on the main.cpp input.
// (Pinocchio and Eigen, which the reference program also uses, are not needed here.)
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "rigidbody.h"

template <typename F>
static double time_us(F &&f) {
    auto t0 = std::chrono::high_resolution_clock::now();
    f();
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count();
}

int main() {
    double q[7] = {0.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0};    // main.cpp:103
    double dq[7] = {0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0};   // main.cpp:104
    double ddq[7] = {1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0};  // main.cpp:105
    Multibody *mb = multibody_new();
    if (!mb) { std::fprintf(stderr, "multibody_new failed\n"); return 1; }
    double *warm = multibody_rnea(mb, q, dq, ddq);  // first call pays model upload / JIT
    std::free(warm);
    double *tau = nullptr;
    double us = time_us([&] { tau = multibody_rnea(mb, q, dq, ddq); });
    double *J = multibody_jac(mb, q);
    double *pos = multibody_fwd_kin(mb, q);
    double *H = multibody_crba(mb, q);
    if (!tau || !J || !pos || !H) { std::fprintf(stderr, "query failed\n"); return 1; }
    std::printf("rnea_us %.1f\n", us);
    std::printf("tau");
    for (int i = 0; i < 7; ++i) std::printf(" %.17g", tau[i]);
    std::printf("\npos");
    for (int i = 0; i < 3; ++i) std::printf(" %.17g", pos[i]);
    std::printf("\njac");
    for (int i = 0; i < 42; ++i) std::printf(" %.17g", J[i]);  // J[6*i + j], main.cpp:76-80
    std::printf("\ncrba");
    for (int i = 0; i < 49; ++i) std::printf(" %.17g", H[i]);  // H[i + 7*j], main.cpp:90-95
    std::printf("\n");
    std::free(tau); std::free(J); std::free(pos); std::free(H);
    multibody_free(mb);
    return 0;
}
