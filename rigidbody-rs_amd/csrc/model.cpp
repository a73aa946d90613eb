// model.cpp -- see model.hpp.
#include "model.hpp"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "urdf.hpp"

namespace rbamd {

void quat_from_scaled_axis(const double v[3], double out[4]) {
    // nalgebra UnitQuaternion::from_scaled_axis = Quaternion::from_imag(v / 2).exp(),
    // identity when |v/2|^2 <= eps^2 (Quaternion::exp_eps).
    const double h0 = v[0] / 2.0, h1 = v[1] / 2.0, h2 = v[2] / 2.0;
    const double nn = h0 * h0 + h1 * h1 + h2 * h2;
    if (nn <= DBL_EPSILON * DBL_EPSILON) {
        out[0] = out[1] = out[2] = 0.0;
        out[3] = 1.0;
        return;
    }
    const double n = std::sqrt(nn);
    const double s = std::sin(n) / n;
    out[0] = h0 * s;
    out[1] = h1 * s;
    out[2] = h2 * s;
    out[3] = std::cos(n);
}

void quat_to_matrix(const double q[4], double R[9]) {
    const double i = q[0], j = q[1], k = q[2], w = q[3];
    const double ww = w * w, ii = i * i, jj = j * j, kk = k * k;
    const double ij = i * j * 2.0, wk = w * k * 2.0, wj = w * j * 2.0;
    const double ik = i * k * 2.0, jk = j * k * 2.0, wi = w * i * 2.0;
    R[0] = ww + ii - jj - kk; R[1] = ij - wk;           R[2] = wj + ik;
    R[3] = wk + ij;           R[4] = ww - ii + jj - kk; R[5] = jk - wi;
    R[6] = ik - wj;           R[7] = wi + jk;           R[8] = ww - ii - jj + kk;
}

void rotation_from_euler(double r, double p, double y, double R[9]) {
    // nalgebra Rotation3::from_euler_angles(roll, pitch, yaw) = Rz(yaw) Ry(pitch) Rx(roll)
    const double sr = std::sin(r), cr = std::cos(r);
    const double sp = std::sin(p), cp = std::cos(p);
    const double sy = std::sin(y), cy = std::cos(y);
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

void rotation_scaled_axis(const double R[9], double out[3]) {
    // nalgebra Rotation3::scaled_axis: axis() = normalise(skew part) or None, * angle()
    const double a0 = R[7] - R[5], a1 = R[2] - R[6], a2 = R[3] - R[1];
    const double n = std::sqrt(a0 * a0 + a1 * a1 + a2 * a2);
    if (!(n > DBL_EPSILON)) {
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    double c = (R[0] + R[4] + R[8] - 1.0) / 2.0;
    c = c > 1.0 ? 1.0 : (c < -1.0 ? -1.0 : c);
    const double ang = std::acos(c);
    out[0] = a0 / n * ang;
    out[1] = a1 / n * ang;
    out[2] = a2 / n * ang;
}

void quat_from_matrix(const double R[9], double q[4]) {
    // Shepperd: branch on the largest of (trace, diagonal) for a well-conditioned sqrt; w >= 0
    const double tr = R[0] + R[4] + R[8];
    double i, j, k, w;
    if (tr > 0.0) {
        const double s = std::sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s; i = (R[7] - R[5]) / s; j = (R[2] - R[6]) / s; k = (R[3] - R[1]) / s;
    } else if (R[0] > R[4] && R[0] > R[8]) {
        const double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2.0;
        w = (R[7] - R[5]) / s; i = 0.25 * s; j = (R[1] + R[3]) / s; k = (R[2] + R[6]) / s;
    } else if (R[4] > R[8]) {
        const double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2.0;
        w = (R[2] - R[6]) / s; i = (R[1] + R[3]) / s; j = 0.25 * s; k = (R[5] + R[7]) / s;
    } else {
        const double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2.0;
        w = (R[3] - R[1]) / s; i = (R[2] + R[6]) / s; j = (R[5] + R[7]) / s; k = 0.25 * s;
    }
    double nrm = std::sqrt(i * i + j * j + k * k + w * w);
    if (w < 0.0) nrm = -nrm;
    q[0] = i / nrm; q[1] = j / nrm; q[2] = k / nrm; q[3] = w / nrm;
}

namespace {

// 3x3 helpers (row-major) for the host-side model build.
void mat_mul(const double A[9], const double B[9], double C[9]) {
    double T[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            T[3 * r + c] = A[3 * r + 0] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
    std::memcpy(C, T, sizeof T);
}
void mat_t(const double A[9], double T[9]) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[3 * c + r] = A[3 * r + c];
}
void mat_vec(const double A[9], const double v[3], double o[3]) {
    double t[3];
    for (int r = 0; r < 3; ++r) t[r] = A[3 * r + 0] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
    std::memcpy(o, t, sizeof t);
}
bool is_identity(const double R[9]) {
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    return std::memcmp(R, I, sizeof I) == 0;
}
bool axis_is_z(const double a[3]) { return std::fabs(a[0]) <= 1e-12 && std::fabs(a[1]) <= 1e-12 && a[2] > 0.0; }

// A rotation R_a with R_a e_z = a (unit): exactly the identity for +z, pi about x for -z,
// else Rodrigues about e_z x a.
void axis_frame(const double a[3], double Ra[9]) {
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (axis_is_z(a)) {
        std::memcpy(Ra, I, sizeof I);
        return;
    }
    const double k[3] = {-a[1], a[0], 0.0};  // e_z x a, |k| = sin
    const double s2 = k[0] * k[0] + k[1] * k[1];
    const double c = a[2];
    if (s2 <= 1e-24) {  // a = -z
        const double F[9] = {1, 0, 0, 0, -1, 0, 0, 0, -1};
        std::memcpy(Ra, F, sizeof F);
        return;
    }
    const double K[9] = {0.0, -k[2], k[1], k[2], 0.0, -k[0], -k[1], k[0], 0.0};
    double K2[9];
    mat_mul(K, K, K2);
    const double f = (1.0 - c) / s2;
    for (int e = 0; e < 9; ++e) Ra[e] = I[e] + K[e] + f * K2[e];
}

// Inertia::from_com (inertia.rs:21-35): I_o = I_c + (m [c]x) [c]x^T
void inertia_about_origin(double mass, const double c[3], const double ic[9], double io[9]) {
    const double C[9] = {0.0, -c[2], c[1], c[2], 0.0, -c[0], -c[1], c[0], 0.0};
    double mC[9];
    for (int k = 0; k < 9; ++k) mC[k] = mass * C[k];
    for (int r = 0; r < 3; ++r)
        for (int col = 0; col < 3; ++col) {
            // (mC) * C^T : sum_k mC[r][k] * C[col][k]
            double s = mC[3 * r + 0] * C[3 * col + 0];
            s += mC[3 * r + 1] * C[3 * col + 1];
            s += mC[3 * r + 2] * C[3 * col + 2];
            io[3 * r + col] = ic[3 * r + col] + s;
        }
}

LinkModel link_from_urdf(const RawJoint &rj) {
    LinkModel L{};
    const double *a = rj.joint.axis;
    const double an = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(an > 0.0)) throw std::runtime_error("joint '" + rj.joint.name + "' has a zero axis");
    for (int k = 0; k < 3; ++k) L.axis[k] = a[k] / an;
    double R[9], sa[3];
    rotation_from_euler(rj.joint.rpy[0], rj.joint.rpy[1], rj.joint.rpy[2], R);
    rotation_scaled_axis(R, sa);
    quat_from_scaled_axis(sa, L.pq);
    std::memcpy(L.pt, rj.joint.xyz, sizeof L.pt);
    L.mass = rj.link.mass;
    std::memcpy(L.com, rj.link.com, sizeof L.com);
    const double *J = rj.link.inertia6;
    const double ic[9] = {J[0], J[1], J[2], J[1], J[3], J[4], J[2], J[4], J[5]};
    std::memcpy(L.icom, ic, sizeof ic);
    inertia_about_origin(L.mass, L.com, L.icom, L.io);
    L.lower = rj.joint.lower;
    L.upper = rj.joint.upper;
    L.velocity = rj.joint.velocity;
    L.effort = rj.joint.effort;
    return L;
}

}  // namespace

namespace {

// Pose of a child frame in its parent: x_parent = R x_child + t.
struct Frame {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double t[3] = {0, 0, 0};
};
Frame compose(const Frame &a, const Frame &b) {
    Frame o;
    mat_mul(a.R, b.R, o.R);
    mat_vec(a.R, b.t, o.t);
    for (int k = 0; k < 3; ++k) o.t[k] += a.t[k];
    return o;
}
Frame joint_origin(const UrdfJoint &j) {
    Frame f;
    rotation_from_euler(j.rpy[0], j.rpy[1], j.rpy[2], f.R);
    std::memcpy(f.t, j.xyz, sizeof f.t);
    return f;
}

// Rigid body accumulated about its own frame origin.
struct Body {
    double mass = 0.0, h[3] = {0, 0, 0}, io[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    void add(const UrdfLink &L, const Frame &T) {
        double Rin[9], Rt[9], ic[9], tmp[9];
        const double *J = L.inertia6;
        const double il[9] = {J[0], J[1], J[2], J[1], J[3], J[4], J[2], J[4], J[5]};
        rotation_from_euler(L.com_rpy[0], L.com_rpy[1], L.com_rpy[2], Rin);
        mat_mul(T.R, Rin, Rin);  // inertial frame -> body frame
        mat_t(Rin, Rt);
        mat_mul(Rin, il, tmp);
        mat_mul(tmp, Rt, ic);
        double c[3];
        mat_vec(T.R, L.com, c);
        for (int k = 0; k < 3; ++k) c[k] += T.t[k];
        double io_l[9];
        inertia_about_origin(L.mass, c, ic, io_l);
        for (int k = 0; k < 9; ++k) io[k] += io_l[k];
        for (int k = 0; k < 3; ++k) h[k] += L.mass * c[k];
        mass += L.mass;
    }
    void to_link(LinkModel &L) const {
        L.mass = mass;
        for (int k = 0; k < 3; ++k) L.com[k] = mass > 0.0 ? h[k] / mass : 0.0;
        std::memcpy(L.io, io, sizeof L.io);
        // I_c = I_o - m [c]x [c]x^T
        double zero[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, P[9];
        inertia_about_origin(mass, L.com, zero, P);
        for (int k = 0; k < 9; ++k) L.icom[k] = io[k] - P[k];
    }
};

bool movable(const std::string &type) {
    return type == "revolute" || type == "continuous" || type == "prismatic";
}

// kModelUrdfTree reading (see model.hpp).  Links are numbered depth-first (preorder): a
// body's movable child joints in the order a stack walk of its fixed subtree meets them
// (each link's joints in document order), so parent indices are always smaller.  The same
// numbering as oracle/urdf_model.py model_frames_from_urdf_tree.
class TreeReader {
  public:
    explicit TreeReader(const UrdfRobot &robot) : robot_(robot) {}

    Model read(bool floating) {
        std::vector<int> as_child(robot_.links.size(), 0);
        for (const UrdfJoint &j : robot_.joints) {
            link_index(j.parent);
            as_child[link_index(j.child)]++;
        }
        int root = -1;
        for (size_t k = 0; k < robot_.links.size(); ++k) {
            if (as_child[k] > 1) throw std::runtime_error("link '" + robot_.links[k].name + "' has several parents");
            if (as_child[k] == 0) {
                if (root >= 0) throw std::runtime_error("URDF has several root links");
                root = (int)k;
            }
        }
        if (root < 0) throw std::runtime_error("URDF has no root link");
        Body root_body;
        std::vector<Child> kids = body(root, &root_body);
        int base = -1;
        if (floating) {
            // virtual joints: prismatic x, y, z (world axes), revolute z, y, x (yaw, pitch,
            // roll); the root body rides on the last one.  Limits shape test inputs only.
            static const double ax[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 1}, {0, 1, 0}, {1, 0, 0}};
            static const double lim[6][3] = {{-1, 1, 1}, {-1, 1, 1}, {-1, 1, 1},
                                             {-M_PI, M_PI, 2}, {-1.2, 1.2, 2}, {-M_PI, M_PI, 2}};
            for (int k = 0; k < 6; ++k) {
                LinkModel L{};
                std::memcpy(L.axis, ax[k], sizeof L.axis);
                L.pq[3] = 1.0;
                L.lower = lim[k][0];
                L.upper = lim[k][1];
                L.velocity = lim[k][2];
                L.effort = 1000.0;
                L.parent = k - 1;
                L.type = k < 3 ? kJointPrismatic : kJointRevolute;
                m_.links.push_back(L);
            }
            root_body.to_link(m_.links[5]);
            base = 5;
        }
        for (const Child &c : kids) visit(c, base);
        return std::move(m_);
    }

  private:
    struct Child {
        const UrdfJoint *joint;
        Frame frame;  // joint origin in the parent body's frame
    };

    int link_index(const std::string &name) const {
        for (size_t k = 0; k < robot_.links.size(); ++k)
            if (robot_.links[k].name == name) return (int)k;
        throw std::runtime_error("joint refers to unknown link '" + name + "'");
    }

    // Link `root` plus its fixed-joint subtree, accumulated into *out; returns its movable
    // child joints.
    std::vector<Child> body(int root, Body *out) const {
        std::vector<Child> kids;
        std::vector<std::pair<int, Frame>> stack{{root, Frame{}}};
        while (!stack.empty()) {
            const auto [ln, T] = stack.back();
            stack.pop_back();
            out->add(robot_.links[ln], T);
            for (const UrdfJoint &j : robot_.joints) {
                if (j.parent != robot_.links[ln].name) continue;
                if (j.mimic) throw std::runtime_error("mimic joint '" + j.name + "' is not supported");
                const Frame Tj = compose(T, joint_origin(j));
                if (j.type == "fixed") {
                    stack.push_back({link_index(j.child), Tj});
                } else if (movable(j.type)) {
                    kids.push_back({&j, Tj});
                } else {
                    throw std::runtime_error("joint '" + j.name + "' of type '" + j.type + "' is not supported");
                }
            }
        }
        return kids;
    }

    void visit(const Child &c, int parent) {
        const UrdfJoint &j = *c.joint;
        LinkModel L{};
        const double *a = j.axis;
        const double an = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (!(an > 0.0)) throw std::runtime_error("joint '" + j.name + "' has a zero axis");
        for (int k = 0; k < 3; ++k) L.axis[k] = a[k] / an;
        quat_from_matrix(c.frame.R, L.pq);
        std::memcpy(L.pt, c.frame.t, sizeof L.pt);
        L.lower = j.lower;
        L.upper = j.upper;
        L.velocity = j.velocity;
        L.effort = j.effort;
        L.parent = parent;
        L.type = j.type == "prismatic" ? kJointPrismatic : kJointRevolute;
        const int idx = (int)m_.links.size();
        m_.links.push_back(L);
        Body b;
        const std::vector<Child> kids = body(link_index(j.child), &b);
        b.to_link(m_.links[idx]);
        for (const Child &k : kids) visit(k, idx);
    }

    const UrdfRobot &robot_;
    Model m_;
};

}  // namespace

Model Model::from_urdf_text(const std::string &xml, unsigned flags) {
    if (flags & ~kModelFlagsAll) throw std::runtime_error("unknown model flags");
    if (flags & kModelFloatingBase) flags |= kModelUrdfTree | kModelGeneralAxes;
    UrdfRobot robot = parse_urdf(xml);
    Model m;
    if (flags & kModelUrdfTree) {
        m = TreeReader(robot).read((flags & kModelFloatingBase) != 0);
    } else {
        std::vector<RawJoint> chain = select_chain(robot, &m.pairing_matches_child);
        for (const RawJoint &rj : chain) {
            m.links.push_back(link_from_urdf(rj));
            m.links.back().parent = (int)m.links.size() - 2;  // multibody.rs: a serial chain
        }
    }
    if (m.links.empty()) throw std::runtime_error("URDF has no non-fixed joint");
    m.n = (int)m.links.size();
    m.flags = flags;
    return m;
}

std::vector<double> Model::blob() const {
    std::vector<double> b(kBlobHeader + (size_t)n * kBlobPerLink, 0.0);
    b[0] = kBlobMagic;
    b[1] = 3.0;
    b[2] = (double)n;
    b[3] = pairing_matches_child ? 1.0 : 0.0;
    b[4] = (double)flags;
    for (int i = 0; i < n; ++i) {
        double *p = &b[kBlobHeader + (size_t)i * kBlobPerLink];
        const LinkModel &L = links[i];
        std::memcpy(p + 0, L.axis, 3 * sizeof(double));
        std::memcpy(p + 3, L.pq, 4 * sizeof(double));
        std::memcpy(p + 7, L.pt, 3 * sizeof(double));
        p[10] = L.mass;
        std::memcpy(p + 11, L.com, 3 * sizeof(double));
        std::memcpy(p + 14, L.icom, 9 * sizeof(double));
        std::memcpy(p + 23, L.io, 9 * sizeof(double));
        p[32] = L.lower;
        p[33] = L.upper;
        p[34] = L.velocity;
        p[35] = L.effort;
        p[36] = (double)L.parent;
        p[37] = (double)L.type;
    }
    return b;
}

Model Model::from_blob(const double *b, int64_t len) {
    if (!b || len < kBlobHeader || b[0] != kBlobMagic || b[1] != 3.0)
        throw std::runtime_error("not a rigidbody model blob (version 3)");
    const int n = (int)b[2];
    if (n < 1 || len != kBlobHeader + (int64_t)n * kBlobPerLink)
        throw std::runtime_error("model blob has the wrong length");
    Model m;
    m.n = n;
    m.pairing_matches_child = b[3] != 0.0;
    if (!(b[4] >= 0.0 && b[4] <= (double)kModelFlagsAll && b[4] == (double)(unsigned)b[4]))
        throw std::runtime_error("model blob has bad flags");
    m.flags = (unsigned)b[4];
    m.links.resize(n);
    for (int i = 0; i < n; ++i) {
        const double *p = &b[kBlobHeader + (size_t)i * kBlobPerLink];
        LinkModel &L = m.links[i];
        std::memcpy(L.axis, p + 0, 3 * sizeof(double));
        std::memcpy(L.pq, p + 3, 4 * sizeof(double));
        std::memcpy(L.pt, p + 7, 3 * sizeof(double));
        L.mass = p[10];
        std::memcpy(L.com, p + 11, 3 * sizeof(double));
        std::memcpy(L.icom, p + 14, 9 * sizeof(double));
        std::memcpy(L.io, p + 23, 9 * sizeof(double));
        L.lower = p[32];
        L.upper = p[33];
        L.velocity = p[34];
        L.effort = p[35];
        L.parent = (int)p[36];
        L.type = (int)p[37];
        if (p[36] != (double)L.parent || L.parent < -1 || L.parent >= i || (L.type != kJointRevolute && L.type != kJointPrismatic))
            throw std::runtime_error("model blob has a bad topology");
    }
    return m;
}

bool Model::all_axes_z() const {
    for (const LinkModel &L : links)
        if (std::fabs(L.axis[0]) > 1e-12 || std::fabs(L.axis[1]) > 1e-12 || L.axis[2] <= 0.0)
            return false;
    return true;
}

bool Model::serial_revolute() const {
    for (int i = 0; i < n; ++i)
        if (links[i].parent != i - 1 || links[i].type != kJointRevolute) return false;
    return true;
}

bool Model::axes_supported() const { return (flags & kModelGeneralAxes) != 0 || all_axes_z(); }

double Model::total_mass() const {
    double s = 0.0;
    for (const LinkModel &L : links) s += L.mass;
    return s;
}

namespace {
template <typename T>
std::vector<T> pack(const Model &m) {
    std::vector<T> out((size_t)m.n * kLinkStride + kTailOut, T(0));
    std::vector<double> Ras((size_t)m.n * 9);
    double Rprev[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};  // base frame: no axis change
    for (int i = 0; i < m.n; ++i) {
        const LinkModel &L = m.links[i];
        T *p = &out[(size_t)i * kLinkStride];
        double R[9], Ra[9], pt[3], com[3], io[9];
        static const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        std::memcpy(Rprev, L.parent >= 0 ? &Ras[(size_t)L.parent * 9] : I3, sizeof Rprev);
        quat_to_matrix(L.pq, R);
        axis_frame(L.axis, Ra);
        std::memcpy(&Ras[(size_t)i * 9], Ra, sizeof Ra);
        std::memcpy(pt, L.pt, sizeof pt);
        std::memcpy(com, L.com, sizeof com);
        std::memcpy(io, L.io, sizeof io);
        if (!is_identity(Rprev) || !is_identity(Ra)) {  // general axis: frame change
            double Pt[9], At[9], tmp[9];
            mat_t(Rprev, Pt);
            mat_t(Ra, At);
            mat_mul(Pt, R, tmp);
            mat_mul(tmp, Ra, R);
            mat_vec(Pt, L.pt, pt);
            mat_vec(At, L.com, com);
            mat_mul(At, L.io, tmp);
            mat_mul(tmp, Ra, io);
        }
        for (int k = 0; k < 9; ++k) p[kE0 + k] = (T)R[k];
        for (int k = 0; k < 3; ++k) p[kP + k] = (T)pt[k];
        p[kM] = (T)L.mass;
        for (int k = 0; k < 3; ++k) p[kH + k] = (T)(L.mass * com[k]);
        p[kIo + 0] = (T)io[0];
        p[kIo + 1] = (T)io[1];
        p[kIo + 2] = (T)io[2];
        p[kIo + 3] = (T)io[4];
        p[kIo + 4] = (T)io[5];
        p[kIo + 5] = (T)io[8];
        p[kParent] = (T)L.parent;
        p[kType] = (T)L.type;
    }
    std::memcpy(Rprev, &Ras[(size_t)(m.n - 1) * 9], sizeof Rprev);  // the last link's axis frame
    // Jacobian start rotation: R_a of the last link, transposed (kinematics.hip jac_kernel)
    T *tail = &out[(size_t)m.n * kLinkStride];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) tail[3 * r + c] = (T)Rprev[3 * c + r];
    return out;
}
}  // namespace

std::vector<float> Model::pack_f32() const { return pack<float>(*this); }
std::vector<double> Model::pack_f64() const { return pack<double>(*this); }

}  // namespace rbamd
