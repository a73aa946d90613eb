// layout.hpp -- packed per-link model constants shared by host (model.cpp) and device.
#pragma once

namespace rbamd {

// Scalars per link in the device constant block.
constexpr int kLinkStride = 24;
// Offsets inside one link's block.
enum : int {
    kE0 = 0,    // parent rotation matrix R_p, row-major (9)
    kP = 9,     // parent translation p (3)
    kM = 12,    // mass
    kH = 13,    // first mass moment h = m * com (3)
    kIo = 16,   // inertia about the link origin, symmetric: xx xy xz yy yz zz (6)
    kParent = 22,  // parent link index (-1: base) -- informational, kernels take topology
    kType = 23,    // joint type (0 revolute, 1 prismatic)  at compile time (jit.cpp)
};

// After the n link blocks: kTailOut scalars, the rotation R0 (row-major) that starts the
// Jacobian's leaf->root accumulation -- identity for the reference's z-axis chains; the
// last link's axis-frame change transposed for general axes (model.cpp pack).
constexpr int kTailOut = 9;

// Base acceleration: the reference's fictitious-gravity trick, +9.81 along base z
// (multibody.rs:117-120).
constexpr double kGravity = 9.81;

}  // namespace rbamd
