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

namespace {

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

Model Model::from_urdf_text(const std::string &xml) {
    UrdfRobot robot = parse_urdf(xml);
    Model m;
    std::vector<RawJoint> chain = select_chain(robot, &m.pairing_matches_child);
    if (chain.empty()) throw std::runtime_error("URDF has no non-fixed joint");
    for (const RawJoint &rj : chain) m.links.push_back(link_from_urdf(rj));
    m.n = (int)m.links.size();
    return m;
}

std::vector<double> Model::blob() const {
    std::vector<double> b(kBlobHeader + (size_t)n * kBlobPerLink, 0.0);
    b[0] = kBlobMagic;
    b[1] = 1.0;
    b[2] = (double)n;
    b[3] = pairing_matches_child ? 1.0 : 0.0;
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
    }
    return b;
}

Model Model::from_blob(const double *b, int64_t len) {
    if (!b || len < kBlobHeader || b[0] != kBlobMagic || b[1] != 1.0)
        throw std::runtime_error("not a rigidbody model blob");
    const int n = (int)b[2];
    if (n < 1 || len != kBlobHeader + (int64_t)n * kBlobPerLink)
        throw std::runtime_error("model blob has the wrong length");
    Model m;
    m.n = n;
    m.pairing_matches_child = b[3] != 0.0;
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
    }
    return m;
}

bool Model::all_axes_z() const {
    for (const LinkModel &L : links)
        if (std::fabs(L.axis[0]) > 1e-12 || std::fabs(L.axis[1]) > 1e-12 || L.axis[2] <= 0.0)
            return false;
    return true;
}

double Model::total_mass() const {
    double s = 0.0;
    for (const LinkModel &L : links) s += L.mass;
    return s;
}

namespace {
template <typename T>
std::vector<T> pack(const Model &m) {
    std::vector<T> out((size_t)m.n * kLinkStride, T(0));
    for (int i = 0; i < m.n; ++i) {
        const LinkModel &L = m.links[i];
        T *p = &out[(size_t)i * kLinkStride];
        double R[9];
        quat_to_matrix(L.pq, R);
        for (int k = 0; k < 9; ++k) p[kE0 + k] = (T)R[k];
        for (int k = 0; k < 3; ++k) p[kP + k] = (T)L.pt[k];
        p[kM] = (T)L.mass;
        for (int k = 0; k < 3; ++k) p[kH + k] = (T)(L.mass * L.com[k]);
        p[kIo + 0] = (T)L.io[0];
        p[kIo + 1] = (T)L.io[1];
        p[kIo + 2] = (T)L.io[2];
        p[kIo + 3] = (T)L.io[4];
        p[kIo + 4] = (T)L.io[5];
        p[kIo + 5] = (T)L.io[8];
    }
    return out;
}
}  // namespace

std::vector<float> Model::pack_f32() const { return pack<float>(*this); }
std::vector<double> Model::pack_f64() const { return pack<double>(*this); }

}  // namespace rbamd
