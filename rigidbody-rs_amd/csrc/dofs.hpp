// dofs.hpp -- chain lengths with a fully unrolled kernel instantiation.
// The recursion over links is unrolled at compile time so every per-link quantity
// stays in registers; each DOF value below is one instantiation per kernel family.
#pragma once

#define RB_FOR_EACH_DOF(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(12) X(16) X(30)

namespace rbamd {
namespace dev {
constexpr int kBlock = 256;
inline unsigned grid_for(unsigned B) { return (B + kBlock - 1) / kBlock; }
}  // namespace dev
}  // namespace rbamd
