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
enum class JitKind : int { Rnea = 0, Fd = 1, Crba = 2, Rollout = 3, FwdKin = 4, Jac = 5 };

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t function = nullptr;       // one configuration per lane (any layout)
    hipFunction_t tile_function = nullptr;  // LDS-tiled, 16-byte global accesses (aligned SoA)
    bool stream = false;        // grid-stride form: launch a resident-sized grid
    int pack = 1;               // configurations per lane (2: paired fp32 lanes, 512 per block)
    int tiles = 1;              // 256-configuration tiles per workgroup (256 x tiles threads)
    unsigned resident = 0;      // resident blocks (occupancy x CUs) for the stream form
    std::string error;          // non-empty when compilation failed
};

bool jit_enabled();

// The LDS-tiled kernel form is generated when the 3N-row input tile fits in 48 KiB.
bool jit_tile_ok(int n, bool f64);

// Generated HIP source for one specialised kernel (exposed for tests / inspection).
// pack: configurations per lane, 0 = the jit_pack policy.
std::string jit_source(const Model &m, JitKind kind, bool f64, bool fast, bool stream, int pack = 0);

// Non-temporal access bits of `kind`'s JIT source, and the cache-key suffix of every
// tuning value that changes the source (tuning.hpp).
int jit_nt(JitKind kind);
bool jit_opaque(JitKind kind, bool f64, int n);
int jit_waves(JitKind kind, bool f64, int n);
// Configurations per lane of `kind`'s lane kernel (tuning `pack`): 2 = paired fp32 lanes.
int jit_pack(JitKind kind, bool f64, int n, bool stream);
// 256-configuration tiles per workgroup of `kind`'s lane kernel (tuning rnea_tiles).
int jit_tiles(JitKind kind, int pack, bool stream);
std::string jit_tag(JitKind kind, bool f64, int n);

// hipRTC compilation only (no device needed): fills `code` with the code object.
bool jit_compile(const Model &m, JitKind kind, bool f64, bool fast, bool stream, const std::string &arch,
                 std::vector<char> *code, std::string *error, int pack = 0);

// Compiles and loads the kernel on the current device.  Never throws.
JitKernel jit_build(const Model &m, JitKind kind, bool f64, bool fast, bool stream, int pack = 0);

}  // namespace rbamd
