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

constexpr int kBlobHeader = 5;    // magic, version, n, index-pairing flag, model flags
constexpr int kBlobPerLink = 38;  // see Model::blob
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
    // Kinematic tree (beyond the reference's serial chain): parent link
    // index (-1 = the fixed base; always < this link's index) and joint type.
    int parent = -1;
    int type = 0;  // kJointRevolute / kJointPrismatic
};

enum : int { kJointRevolute = 0, kJointPrismatic = 1 };

// Model-reading flags (rigidbody_batch.h RB_MODEL_*).
enum : unsigned {
    // Any revolute axis, with the motion subspace S = (axis, 0) -- the reference hard-codes
    // z (multibody.rs:130-138) and is only consistent for z axes.  Identical results for
    // z-axis chains.  Implemented by a constant per-link frame change at pack time.
    kModelGeneralAxes = 1u,
    // Physical URDF tree instead of the reference's index pairing (multibody.rs:70):
    // follow joint parent/child names from the root link, merge fixed joints (their
    // child bodies join the parent body, their origins compose into the next joint),
    // honour the inertial-origin rpy.  Kinematic trees (links numbered depth-first, parents
    // first) and revolute / continuous / prismatic joints; mimic joints are rejected.
    kModelUrdfTree = 2u,
    // Free-floating root: six massless virtual joints (prismatic x, y, z; revolute z, y, x)
    // between the world and the root body.  Implies kModelUrdfTree | kModelGeneralAxes.
    kModelFloatingBase = 4u,
    kModelFlagsAll = 7u,
};

struct Model {
    int n = 0;
    std::vector<LinkModel> links;
    bool pairing_matches_child = true;
    unsigned flags = 0;

    // throws std::runtime_error
    static Model from_urdf_text(const std::string &xml, unsigned flags = 0);
    static Model from_blob(const double *blob, int64_t len);
    std::vector<double> blob() const;

    bool all_axes_z() const;
    // The reference's topology: parent(i) = i - 1 and every joint revolute.  Only such
    // models run on the precompiled generic kernels; trees and prismatic joints need the
    // model-specialised (hipRTC) ones.
    bool serial_revolute() const;
    // Every axis usable under `flags`: +z always, any direction with kModelGeneralAxes.
    bool axes_supported() const;
    double total_mass() const;

    // Device constants: n * kLinkStride scalars laid out per link as layout.hpp says, then
    // kTailOut.  A link whose axis is not +z is re-expressed in a frame whose z is its
    // axis (R_a e_z = axis): R_p' = R_a,parent^T R_p R_a, p' = R_a,parent^T p (parent = the
    // link's tree parent, identity for the base),
    // c' = R_a^T c, I' = R_a^T I R_a -- so the kernels' z-joint code is exact for any axis.
    std::vector<float> pack_f32() const;
    std::vector<double> pack_f64() const;
};

// nalgebra-equivalent helpers (also used for unit tests through the C ABI-free path).
void quat_from_scaled_axis(const double v[3], double out[4]);
void quat_to_matrix(const double q[4], double R[9]);
void rotation_from_euler(double r, double p, double y, double R[9]);
void rotation_scaled_axis(const double R[9], double out[3]);
void quat_from_matrix(const double R[9], double q[4]);

}  // namespace rbamd
