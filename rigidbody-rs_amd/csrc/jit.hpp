// jit.hpp -- model-specialised kernels compiled at model-load time with hipRTC.
//
// The precompiled kernels read the model's per-link constants from LDS, so every
// rotation entry and offset costs an FMA even when it is 0 or +-1.  URDF joint frames
// are usually signed axis permutations (rpy in multiples of pi/2) with sparse offsets;
// compiling the SAME device code (rnea_body.hip.hpp) against the model as a constexpr
// array lets the compiler fold those constants away (FR3 RNEA: ~1090 -> see DESIGN.md).
// Rotation/offset entries within 1e-14 of 0 or +-1 are snapped to exactly those values
// (the reference's own quaternion->matrix round trip leaves 1e-16 residues there), and
// the module is compiled with -ffinite-math-only -fno-signed-zeros so 0*x and 1*x fold.
//
// Any hipRTC failure leaves the precompiled generic kernel in charge (still on the GPU);
// RB_JIT=0 (or rb_set_tuning("jit", 0)) disables the path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "model.hpp"

namespace rbamd {

// FwdKin / Jac: built only for models the precompiled kinematics kernels cannot express
// (kinematic trees, prismatic joints -- Model::serial_revolute() false).
// RneaFd: inverse + forward dynamics of the same (q, qd) in one launch (fdh_body.hip.hpp
// fdh_idfd_eval), for models on the mass-matrix forward dynamics (jit_fd_form 2).
enum class JitKind : int { Rnea = 0, Fd = 1, Crba = 2, Rollout = 3, FwdKin = 4, Jac = 5, RneaFd = 6 };
constexpr int kJitKinds = 7;

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t function = nullptr;  // the lane kernel (any layout)
    int pack = 1;                      // configurations per lane (2: paired fp32 lanes, 512 per block)
    int seq_tail = 0;                  // pack 3: trailing tiles run one per lane (tuning seq_tail)
    unsigned block = 256;              // threads per block
    std::string error;                 // non-empty when compilation failed
};

bool jit_enabled();

// Generated HIP source for one specialised kernel (exposed for tests / inspection).
// pack: configurations per lane, 0 = the jit_pack policy.
// tail: sequential-pair RNEA only -- percent of the launch's tiles run one per lane (0 none).
// nt: the non-temporal load / store bits compiled in (RB_NT); -1 = jit_nt(kind).
// waves: amdgpu_waves_per_eu target of the kernel; -1 = the policy (jit_waves and the per-form
// rules in jit_source).  jit_compile may rebuild with a 2-wave target (occupancy cliff, below).
std::string jit_source(const Model &m, JitKind kind, bool f64, bool fast, int pack = 0, int tail = 0, int nt = -1,
                       int waves = -1);

// Unified VGPR count (arch VGPRs + AGPRs) of a code object's kernel, from its AMDGPU metadata;
// -1 if not found.
int code_vgprs(const std::vector<char> &code);

// Non-temporal access bits of `kind`'s JIT source, and the cache-key suffix of every
// tuning value that changes the source (tuning.hpp).
int jit_nt(JitKind kind);
bool jit_opaque(JitKind kind, bool f64, int n);
int jit_waves(JitKind kind, bool f64, int n);
// Configurations per lane of `kind`'s lane kernel (tuning `pack`): 2 = paired fp32 lanes.
int jit_pack(JitKind kind, bool f64, int n);
std::string jit_tag(JitKind kind, bool f64, int n);
// Forward-dynamics algorithm for this model (tuning fd_form): 2 = mass-matrix method
// (fdh_body.hip.hpp), 1 = Articulated-Body Algorithm (aba_body.hip.hpp).
int jit_fd_form(const Model &m, JitKind kind = JitKind::Fd);
// The lane form a kernel of this model really takes for the requested pack (0 = policy).
int jit_model_pack(const Model &m, JitKind kind, bool f64, int pack_req);
// Percent of a sequential-pair RNEA launch's tiles run one per lane for this layout (tuning
// seq_tail; auto: 75 for the tiled layout, 0 for SoA).
int jit_seq_tail(bool tiled);

// hipRTC compilation only (no device needed): fills `code` with the code object.  Occupancy
// cliff: a kernel built without an occupancy target that lands just past 256 registers (one
// wave per SIMD, <= 16 over) is rebuilt with a 2-wave target -- a few spilled values cost less
// than half the SIMD's waves (the 9-joint tree's fp64 RNEA: 258 registers; 65.0 vs 92.9 us at
// 2^20 with 12 B of scratch; 234 registers at the first build once the kernel arguments are
// preloaded, tuning.hpp kernarg_preload).
// final_src (optional): the source of the code object returned -- the occupancy-cliff rebuild's
// when that rule applied (multibody_jit_source_ex reports this one).
bool jit_compile(const Model &m, JitKind kind, bool f64, bool fast, const std::string &arch,
                 std::vector<char> *code, std::string *error, int pack = 0, int tail = 0,
                 int nt = -1, std::string *final_src = nullptr);

// Compiles and loads the kernel on the current device.  Never throws.
JitKernel jit_build(const Model &m, JitKind kind, bool f64, bool fast, int pack = 0, int tail = 0, int nt = -1);

}  // namespace rbamd
