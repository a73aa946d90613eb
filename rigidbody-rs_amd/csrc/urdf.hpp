// urdf.hpp -- minimal XML reader + URDF model extraction (host, run once per model).
//
// Restates what the reference gets from xurdf 0.2.5 (Cargo.lock:618-629) and uses in
// Multibody::from_urdf (multibody.rs:65-77): the TOP-LEVEL <link>/<joint> children of
// <robot> in document order (joints nested in <transmission>/<gazebo> are not robot
// joints), paired BY INDEX, keeping pairs whose joint type does not contain "fixed".
#pragma once

#include <limits>
#include <string>
#include <vector>

namespace rbamd {

struct XmlNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<XmlNode> children;
    const char *attr(const char *name) const;
    const XmlNode *child(const char *tag) const;
};

// Throws std::runtime_error with a position on malformed input.
XmlNode parse_xml(const std::string &text);

struct UrdfLink {
    std::string name;
    double mass = 0.0;
    double com[3] = {0, 0, 0};      // <inertial><origin xyz>; rpy ignored (joint.rs:66)
    double com_rpy[3] = {0, 0, 0};  // <inertial><origin rpy>: used only by the tree reading
    double inertia6[6] = {0, 0, 0, 0, 0, 0}; // ixx ixy ixz iyy iyz izz
};

struct UrdfJoint {
    std::string name, type, parent, child;
    double xyz[3] = {0, 0, 0};
    double rpy[3] = {0, 0, 0};
    double axis[3] = {1, 0, 0};     // URDF default when <axis> is absent
    static constexpr double kNaN = std::numeric_limits<double>::quiet_NaN();
    double lower = kNaN, upper = kNaN, effort = kNaN, velocity = kNaN;
    bool mimic = false;             // has a <mimic> child
};

struct UrdfRobot {
    std::string name;
    std::vector<UrdfLink> links;
    std::vector<UrdfJoint> joints;
};

UrdfRobot parse_urdf(const std::string &text);

// One revolute joint + its paired link, in chain order.
struct RawJoint {
    UrdfJoint joint;
    UrdfLink link;
};

// multibody.rs:65-77: zip(joints, links) by index, skip "fixed".  Also reports whether
// the index pairing agrees with the physical (joint.child == link.name) pairing.
std::vector<RawJoint> select_chain(const UrdfRobot &robot, bool *pairing_matches_child);

}  // namespace rbamd
