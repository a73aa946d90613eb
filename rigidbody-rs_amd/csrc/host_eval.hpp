// host_eval.hpp -- single-configuration queries on the host (see host_eval.cpp).
#pragma once

#include "model.hpp"

namespace rbamd {

// FMA3 present on this CPU (checked once).
bool host_fma_available();
// Serial revolute chain of a precompiled DOF on an FMA3 host.
bool host_eval_supported(const Model &m);

// `pk` = Model::pack_f64() (the generic kernels' constant block).  Each returns false
// (nothing written) when the model / CPU is not supported; outputs follow the reference ABI
// (lib.rs:15-70): tau[n]; H[n*n] column-major upper triangle, exact-zero lower; pos[3];
// J[6n] column-major, rows [lin; rot].
bool host_rnea(const Model &m, const double *pk, const double *q, const double *qd, const double *qdd, double *tau);
bool host_crba(const Model &m, const double *pk, const double *q, double *H);
bool host_fwd_kin(const Model &m, const double *pk, const double *q, double *pos);
bool host_jac(const Model &m, const double *pk, const double *q, double *J);

}  // namespace rbamd
