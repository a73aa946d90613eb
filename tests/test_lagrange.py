"""Independent physics pin for the RNEA / CRBA semantics: the equations of
motion of 3-link z-axis chains derived symbolically from the Lagrangian (sympy; no spatial
algebra, no recursion) -- L = sum_i 1/2 m_i |v_ci|^2 + 1/2 w_i^T I_ci w_i - m_i g z_ci with the
reference's conventions (joint frame = origin xyz/rpy then Rz(q), nalgebra from_euler_angles =
Rz(y) Ry(p) Rx(r); com inertia in the link frame, inertial rpy ignored, inertia.rs:21-35;
gravity 9.81 along -z, the reference's fictitious base acceleration multibody.rs:117-120) --
against the oracle (oracle/oracle.c) AND the product's own lane bodies through the
single-configuration ABI (csrc/host_eval.cpp).  The reference holds no RNEA outputs, so this
ties both to classical mechanics rather than to a second Featherstone restatement.  CPU only."""
import numpy as np
import pytest

sp = pytest.importorskip("sympy")

G = 9.81


def _rpy(r, p, y):
    cr, sr, cp, s_p, cy, sy = (sp.Float(v) for v in (np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)))
    Rx = sp.Matrix([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = sp.Matrix([[cp, 0, s_p], [0, 1, 0], [-s_p, 0, cp]])
    Rz = sp.Matrix([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz * Ry * Rx


def _lagrangian_dynamics(raw):
    """tau(q, qd, qdd) and M(q) from the Lagrangian, lambdified."""
    n = raw["n"]
    q, qd, qdd = sp.symbols(f"q0:{n}"), sp.symbols(f"qd0:{n}"), sp.symbols(f"qdd0:{n}")
    R, p = sp.eye(3), sp.zeros(3, 1)
    T, V = 0, 0
    for i in range(n):
        p = p + R * sp.Matrix(raw["xyz"][i])
        c, s = sp.cos(q[i]), sp.sin(q[i])
        R = R * _rpy(*raw["rpy"][i]) * sp.Matrix([[c, -s, 0], [s, c, 0], [0, 0, 1]])
        pc = p + R * sp.Matrix(raw["com"][i])
        vc = pc.jacobian(q) * sp.Matrix(qd)
        Rdot = sp.zeros(3, 3)
        for k in range(n):
            Rdot += R.diff(q[k]) * qd[k]
        W = R.T * Rdot  # body angular velocity, skew form
        wb = sp.Matrix([W[2, 1], W[0, 2], W[1, 0]])
        I6 = raw["inertia6"][i]
        Ic = sp.Matrix([[I6[0], I6[1], I6[2]], [I6[1], I6[3], I6[4]], [I6[2], I6[4], I6[5]]])
        m = float(raw["mass"][i])
        T += sp.Rational(1, 2) * m * (vc.T * vc)[0] + sp.Rational(1, 2) * (wb.T * Ic * wb)[0]
        V += m * G * pc[2]
    L = T - V
    dL = [sp.diff(L, v) for v in qd]
    tau = [sum(sp.diff(dL[i], qd[j]) * qdd[j] + sp.diff(dL[i], q[j]) * qd[j] for j in range(n)) - sp.diff(L, q[i])
           for i in range(n)]
    M = [[sp.diff(dL[i], qd[j]) for j in range(n)] for i in range(n)]
    return sp.lambdify((q, qd, qdd), tau, "numpy", cse=True), sp.lambdify((q,), M, "numpy", cse=True)


def _random_chain_urdf(seed):
    """3-link z-axis chain with dense joint frames (rpy not multiples of pi/2) and random
    inertials (positive-definite com inertia)."""
    rng = np.random.default_rng(seed)
    out = ['<robot name="rand3">']
    for k in range(3):
        A = rng.normal(size=(3, 3))
        Ic = A @ A.T * 0.05 + np.eye(3) * 0.02
        com = rng.uniform(-0.1, 0.1, 3)
        out += [f'<link name="l{k}"><inertial><origin xyz="{com[0]} {com[1]} {com[2]}" rpy="0 0 0"/>'
                f'<mass value="{rng.uniform(0.5, 3.0)}"/>'
                f'<inertia ixx="{Ic[0, 0]}" ixy="{Ic[0, 1]}" ixz="{Ic[0, 2]}" iyy="{Ic[1, 1]}" iyz="{Ic[1, 2]}" '
                f'izz="{Ic[2, 2]}"/></inertial></link>']
    for k in range(3):
        xyz, rpy = rng.uniform(-0.3, 0.3, 3), rng.uniform(-1.2, 1.2, 3)
        out += [f'<joint name="j{k}" type="revolute"><origin xyz="{xyz[0]} {xyz[1]} {xyz[2]}" '
                f'rpy="{rpy[0]} {rpy[1]} {rpy[2]}"/><parent link="{"l" + str(k - 1) if k else "base"}"/>'
                f'<child link="l{k}"/><axis xyz="0 0 1"/>'
                f'<limit lower="-3" upper="3" effort="50" velocity="2"/></joint>']
    return "".join(out) + "</robot>"


@pytest.fixture(scope="module")
def models():
    from rigidbody_amd import chains

    return {"fr3_links_1_3": chains.synthetic_chain_urdf(3), "dense_frames": _random_chain_urdf(7)}


@pytest.mark.parametrize("name", ["fr3_links_1_3", "dense_frames"])
def test_rnea_crba_match_lagrangian(name, models, oracle_mod):
    from oracle import urdf_model
    from rigidbody_amd import ffi

    xml = models[name]
    raw = urdf_model.model_raw_from_urdf(xml)
    tau_l, M_l = _lagrangian_dynamics(raw)
    om = oracle_mod.Model(raw)
    mb = ffi.Multibody.from_urdf_string(xml)
    assert mb.single_config_path() == "host"
    rng = np.random.default_rng(3)
    for _ in range(25):
        q, qd, qdd = (rng.uniform(-2.5, 2.5, 3) for _ in range(3))
        want = np.array(tau_l(q, qd, qdd), float)
        M = np.array(M_l(q), float)
        scale = 1 + np.abs(want).max()
        assert np.abs(om.rnea(q, qd, qdd) - want).max() <= 1e-12 * scale
        assert np.abs(mb.rnea(q, qd, qdd) - want).max() <= 1e-12 * scale
        H = om.crba(q)
        Hs = np.triu(H) + np.triu(H, 1).T
        assert np.abs(Hs - M).max() <= 1e-12 * (1 + np.abs(M).max())
        Hg = mb.crba(q)  # the ABI's upper triangle
        assert np.abs(np.triu(Hg) + np.triu(Hg, 1).T - M).max() <= 1e-12 * (1 + np.abs(M).max())
        # forward dynamics: M qdd = tau - bias, with the Lagrangian's own bias
        t = rng.uniform(-20, 20, 3)
        qdd_l = np.linalg.solve(M, t - np.array(tau_l(q, qd, np.zeros(3)), float))
        assert np.abs(om.fd(q, qd, t) - qdd_l).max() <= 1e-10 * (1 + np.abs(qdd_l).max())
