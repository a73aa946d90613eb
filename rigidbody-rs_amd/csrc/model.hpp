// model.hpp -- host-side model (fp64) and its packed device form.
//
// One RevoluteJoint per chain link, as the reference builds them
// (RevoluteJoint::from_xurdf_joint, joint.rs:53-68):
//   axis    = normalise(<axis xyz>)                                   joint.rs:56
//   parent  = Isometry3(xyz, Rotation3::from_euler_angles(rpy).scaled_axis())  57-64
//   body    = Inertia::from_com(mass, inertial xyz, inertia)          66, inertia.rs:21-35
// The nalgebra arithmetic (quaternion from scaled axis, quaternion->matrix, RPY) is
// restated in model.cpp; it runs once per model, off the timed path.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "layout.hpp"

namespace rbamd {

constexpr int kBlobHeader = 4;    // magic, version, n, reserved
constexpr int kBlobPerLink = 36;  // see Model::blob
constexpr double kBlobMagic = 20250224.0;

struct LinkModel {
    double axis[3];
    double pq[4];  // parent rotation quaternion, nalgebra coords (i, j, k, w)
    double pt[3];  // parent translation
    double mass;
    double com[3];
    double icom[9];  // about COM, row-major
    double io[9];    // about link origin, row-major
    double lower, upper, velocity, effort;
};

struct Model {
    int n = 0;
    std::vector<LinkModel> links;
    bool pairing_matches_child = true;

    static Model from_urdf_text(const std::string &xml);  // throws std::runtime_error
    static Model from_blob(const double *blob, int64_t len);
    std::vector<double> blob() const;

    bool all_axes_z() const;
    double total_mass() const;

    // Device constants: n * kLinkStride scalars, laid out per link as the enum above.
    std::vector<float> pack_f32() const;
    std::vector<double> pack_f64() const;
};

// nalgebra-equivalent helpers (also used for unit tests through the C ABI-free path).
void quat_from_scaled_axis(const double v[3], double out[4]);
void quat_to_matrix(const double q[4], double R[9]);
void rotation_from_euler(double r, double p, double y, double R[9]);
void rotation_scaled_axis(const double R[9], double out[3]);

}  // namespace rbamd
