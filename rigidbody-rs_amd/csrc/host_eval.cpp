// host_eval.cpp -- the reference's single-configuration queries on the host CPU.
//
// SURVEY §8(d) config 1 is the reference's CPU path: one configuration per call
// (rigidbody_bindings/src/lib.rs:15-70, timed by main.cpp:69).  A GPU round trip (H2D copy,
// launch, D2H copy, stream sync) costs ~18 us there against ~0.7 us for the CPU recursion,
// so multibody_rnea / _crba / _fwd_kin / _jac evaluate the configuration on the calling
// thread -- with the SAME lane bodies the GPU kernels run (rnea_body / crba_body /
// tree_body .hip.hpp are host+device, RB_HD), instantiated here for the host against the
// packed fp64 model the precompiled kernels stage into LDS.  This is not a fallback: it is
// the single-configuration dispatch (capi.cpp single_dispatch); every batched entry point
// runs on the GPU only.  Serial revolute chains of a precompiled DOF (dofs.hpp) only; tree
// models keep the GPU path (their topology is compiled in by hipRTC).  Needs FMA3 + AVX2 on the host
// (the recursion is written in fused multiply-adds); without it the GPU path serves.
#include "host_eval.hpp"

#include "crba_body.hip.hpp"
#include "dofs.hpp"
#include "kernels.hpp"
#include "rnea_body.hip.hpp"

namespace rbamd {
namespace {

// The reference's serial chain as a full topology policy, so the tree forms of FK / the
// Jacobian (tree_body.hip.hpp) evaluate it: every link is on the last link's path.
template <int N>
struct HostSerialTopo {
    static constexpr bool kSerial = true;
    static constexpr int parent(int j) { return j - 1; }
    static constexpr bool prismatic(int) { return false; }
    static constexpr int last_child(int j) { return j + 1 < N ? j + 1 : -1; }
    static constexpr bool is_ancestor(int a, int i) { return a < i; }
    static constexpr int child_toward(int a, int i) { return a < i ? a + 1 : -1; }
    static constexpr bool on_path(int) { return true; }
};

#define RB_HOST_FMA __attribute__((target("avx2,fma")))

RB_HOST_FMA bool rnea_fma(int n, const double *mdl, const double *q, const double *qd, const double *qdd,
                          double *tau) {
    switch (n) {
#define X(N)                                                                                        \
    case N: {                                                                                       \
        double a[N], b[N], c[N];                                                                    \
        for (int j = 0; j < N; ++j) {                                                               \
            a[j] = q[j];                                                                            \
            b[j] = qd[j];                                                                           \
            c[j] = qdd[j];                                                                          \
        }                                                                                           \
        dev::rnea_eval<double, N, false>(mdl, a, b, c, [&](int j, double v) { tau[j] = v; });       \
        return true;                                                                                \
    }
        RB_FOR_EACH_DOF(X)
#undef X
        default: return false;
    }
}

RB_HOST_FMA bool crba_fma(int n, const double *mdl, const double *q, double *H) {
    switch (n) {
#define X(N)                                                                                        \
    case N: {                                                                                       \
        double a[N];                                                                                \
        for (int j = 0; j < N; ++j) a[j] = q[j];                                                    \
        dev::crba_eval<double, N, false>(mdl, a, [&](int e, double v) { H[e] = v; });               \
        return true;                                                                                \
    }
        RB_FOR_EACH_DOF(X)
#undef X
        default: return false;
    }
}

RB_HOST_FMA bool fwd_kin_fma(int n, const double *mdl, const double *q, double *pos) {
    switch (n) {
#define X(N)                                                                                        \
    case N: {                                                                                       \
        double a[N];                                                                                \
        for (int j = 0; j < N; ++j) a[j] = q[j];                                                    \
        dev::fwd_kin_tree<double, N, false, HostSerialTopo<N>>(mdl, a, [&](int e, double v) { pos[e] = v; }); \
        return true;                                                                                \
    }
        RB_FOR_EACH_DOF(X)
#undef X
        default: return false;
    }
}

RB_HOST_FMA bool jac_fma(int n, const double *mdl, const double *q, double *J) {
    switch (n) {
#define X(N)                                                                                        \
    case N: {                                                                                       \
        double a[N];                                                                                \
        for (int j = 0; j < N; ++j) a[j] = q[j];                                                    \
        dev::jac_tree<double, N, false, HostSerialTopo<N>>(mdl, a, [&](int e, double v) { J[e] = v; }); \
        return true;                                                                                \
    }
        RB_FOR_EACH_DOF(X)
#undef X
        default: return false;
    }
}

}  // namespace

bool host_fma_available() {
    static const bool ok = __builtin_cpu_supports("fma") && __builtin_cpu_supports("avx2");
    return ok;
}

bool host_eval_supported(const Model &m) { return host_fma_available() && m.serial_revolute() && dof_supported(m.n); }

bool host_rnea(const Model &m, const double *pk, const double *q, const double *qd, const double *qdd, double *tau) {
    return host_eval_supported(m) && rnea_fma(m.n, pk, q, qd, qdd, tau);
}

bool host_crba(const Model &m, const double *pk, const double *q, double *H) {
    return host_eval_supported(m) && crba_fma(m.n, pk, q, H);
}

bool host_fwd_kin(const Model &m, const double *pk, const double *q, double *pos) {
    return host_eval_supported(m) && fwd_kin_fma(m.n, pk, q, pos);
}

bool host_jac(const Model &m, const double *pk, const double *q, double *J) {
    return host_eval_supported(m) && jac_fma(m.n, pk, q, J);
}

}  // namespace rbamd
