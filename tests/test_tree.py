"""Kinematic trees, prismatic joints and a floating base (beyond the
reference's serial revolute chain; RB_MODEL_URDF_TREE / RB_MODEL_FLOATING_BASE) -- CPU side.

The reference has none of these, so parity is pinned by two independent restatements:
oracle.c (quaternion / isometry code path, parent array) against the 6x6 Featherstone
tree forms (featherstone6.py), plus physics invariants that need no restatement at all:
  * free fall: with a floating base, qd = 0 and tau = 0, every body falls together --
    qdd = (0, 0, -g, 0, ..., 0) in any configuration;
  * the floating base's translational block of H is the total mass times the identity;
  * rnea(q, qd, fd(q, qd, tau)) = tau and H symmetric positive definite.
The product's C++ tree reading (model.cpp) is checked against the Python one.
"""
import numpy as np
import pytest

G = 9.81


def _models(xml, floating, oracle_mod):
    from oracle import featherstone6, urdf_model

    fr = urdf_model.model_frames_from_urdf_tree(xml, floating=floating)
    return fr, oracle_mod.Model(frames=fr, general=True), featherstone6.Model6(frames=fr, general=True)


def _q(fr, rng):
    from rigidbody_amd import chains

    lim = fr["limits"]
    lo = np.array([(l or {}).get("lower", -np.pi) for l in lim])
    hi = np.array([(l or {}).get("upper", np.pi) for l in lim])
    return lo + (hi - lo) * rng.random(fr["n"])


@pytest.mark.parametrize("floating", [False, True])
def test_tree_oracle_matches_6x6(floating, oracle_mod):
    from rigidbody_amd import chains

    fr, om, m6 = _models(chains.tree_urdf(floating=floating), floating, oracle_mod)
    n = fr["n"]
    assert n == (14 if floating else 9)
    assert list(fr["parent"][:1]) == [-1] and all(fr["parent"][i] < i for i in range(n))
    assert fr["prismatic"].sum() == (4 if floating else 2)
    assert len(set(fr["parent"])) < n  # really branches
    rng = np.random.default_rng(4)
    for _ in range(8):
        q = _q(fr, rng)
        qd, qdd = rng.uniform(-2, 2, (2, n))
        tau = om.rnea(q, qd, qdd)
        assert np.abs(tau - m6.rnea(q, qd, qdd)).max() <= 1e-11 * (1 + np.abs(tau).max())
        H, H6 = om.crba(q), m6.crba(q)
        assert np.all(np.tril(H, -1) == 0.0)
        assert np.abs(np.triu(H) - np.triu(H6)).max() <= 1e-12 * (1 + np.abs(H6).max())
        Hs = np.triu(H) + np.triu(H, 1).T
        assert np.linalg.eigvalsh(Hs).min() > 0
        assert np.abs(om.jac(q) - m6.jac(q)).max() <= 1e-12
        assert np.abs(om.fwd_kin(q) - m6.fwd_kin(q)).max() <= 1e-12
        qdd_fd = om.fd(q, qd, tau)
        assert np.abs(qdd_fd - qdd).max() <= 1e-8 * (1 + np.abs(qdd).max())
        assert np.abs(m6.aba(q, qd, tau) - qdd).max() <= 1e-8 * (1 + np.abs(qdd).max())


def test_tree_structure_zeros(oracle_mod):
    """H couples only ancestor/descendant pairs; J has zero columns off the leaf's path."""
    from rigidbody_amd import chains

    fr, om, _ = _models(chains.tree_urdf(), False, oracle_mod)
    n, par = fr["n"], fr["parent"]

    def anc(i):
        out = set()
        while i >= 0:
            out.add(i)
            i = par[i]
        return out

    q = _q(fr, np.random.default_rng(1))
    H, J = om.crba(q), om.jac(q)
    for i in range(n):
        for j in range(i):
            related = j in anc(i)
            assert (H[j, i] != 0.0) == related, (j, i)
    path = anc(n - 1)
    for i in range(n):
        assert np.any(J[:, i] != 0.0) == (i in path)


def test_floating_base_free_fall(oracle_mod):
    from rigidbody_amd import chains

    fr, om, m6 = _models(chains.tree_urdf(floating=True), True, oracle_mod)
    n = fr["n"]
    rng = np.random.default_rng(9)
    want = np.zeros(n)
    want[2] = -G
    total = fr["mass"].sum()
    for _ in range(6):
        q = _q(fr, rng)
        assert np.abs(om.fd(q, np.zeros(n), np.zeros(n)) - want).max() <= 1e-10
        assert np.abs(m6.aba(q, np.zeros(n), np.zeros(n)) - want).max() <= 1e-10
        H = om.crba(q)
        assert np.abs(np.triu(H[:3, :3]) - np.triu(total * np.eye(3))).max() <= 1e-12 * total
        # gravity compensation: a floating robot at rest needs a force m g up on its base
        tau = om.rnea(q, np.zeros(n), np.zeros(n))
        assert np.abs(tau[:3] - [0.0, 0.0, total * G]).max() <= 1e-10 * total * G


def test_serial_topology_is_bit_identical(oracle_mod, fr3_text):
    """Explicit serial parents reproduce the default (reference) code path bit for bit."""
    from oracle import urdf_model

    fr = urdf_model.model_frames_from_urdf_tree(fr3_text)
    a = oracle_mod.Model(frames=fr)
    fr2 = {k: v for k, v in fr.items() if k not in ("parent", "prismatic")}
    b = oracle_mod.Model(frames=fr2)
    rng = np.random.default_rng(2)
    for _ in range(8):
        q, qd, qdd = rng.uniform(-2, 2, (3, 7))
        assert np.array_equal(a.rnea(q, qd, qdd), b.rnea(q, qd, qdd))
        assert np.array_equal(a.crba_raw(q), b.crba_raw(q))
        assert np.array_equal(a.jac_raw(q), b.jac_raw(q))
        assert np.array_equal(a.fwd_kin(q), b.fwd_kin(q))


@pytest.mark.parametrize("floating", [False, True])
def test_tree_reading_cpp_matches_python(floating, oracle_mod):
    from oracle import urdf_model
    from rigidbody_amd import chains, ffi

    xml = chains.tree_urdf(floating=floating)
    fr = urdf_model.model_frames_from_urdf_tree(xml, floating=floating)
    flags = ffi.FLOATING_BASE if floating else ffi.URDF_TREE | ffi.GENERAL_AXES
    mb = ffi.Multibody.from_urdf_string(xml, flags)
    n = fr["n"]
    assert mb.n == n and mb.flags == (7 if floating else 3)
    par, typ = mb.topology()
    assert np.array_equal(par, fr["parent"]) and np.array_equal(typ, fr["prismatic"])
    L = mb.blob()[5:].reshape(n, 38)
    for i in range(n):
        assert np.abs(oracle_mod.quat_to_matrix(L[i, 3:7]) - fr["Rp"][i]).max() <= 1e-13
        assert np.abs(L[i, 7:10] - fr["p"][i]).max() <= 1e-13
        assert L[i, 0:3] == pytest.approx(fr["axis"][i], abs=1e-15)
        assert L[i, 10] == pytest.approx(fr["mass"][i], rel=1e-15, abs=1e-300)
        assert np.abs(L[i, 11:14] - fr["com"][i]).max() <= 1e-13
        assert np.abs(L[i, 14:23].reshape(3, 3) - fr["icom"][i]).max() <= 1e-13
        assert (L[i, 36], L[i, 37]) == (fr["parent"][i], fr["prismatic"][i])
    lo, hi, vel, eff = mb.limits()
    for i in range(n):
        lim = fr["limits"][i] or {}
        for arr, key in ((lo, "lower"), (hi, "upper"), (vel, "velocity"), (eff, "effort")):
            if key in lim:
                assert arr[i] == pytest.approx(lim[key], rel=1e-15)
    assert mb.total_mass == pytest.approx(fr["mass"].sum(), rel=1e-14)
    mb2 = ffi.Multibody.from_blob(mb.blob())  # the RCCL broadcast path keeps the topology
    assert np.array_equal(mb2.topology()[0], par) and np.array_equal(mb2.topology()[1], typ)


@pytest.mark.parametrize("floating", [False, True])
def test_tree_kernels_compile_for_gfx950(floating):
    """hipRTC builds every model-specialised tree kernel (no device needed)."""
    from rigidbody_amd import chains, ffi

    flags = ffi.FLOATING_BASE if floating else ffi.URDF_TREE | ffi.GENERAL_AXES
    mb = ffi.Multibody.from_urdf_string(chains.tree_urdf(floating=floating), flags)
    for kind in ("rnea", "fd", "crba", "rollout", "fwd_kin", "jac"):
        for f64 in ((True,) if kind in ("fwd_kin", "jac") else (False, True)):
            src = mb.jit_source(f64, kind)
            assert "struct Topo" in src and "kSerial = false" in src
            assert mb.jit_compile(f64=f64, kind=kind) > 0
    # a serial revolute chain keeps the tuned serial code path
    assert "using Topo = rbamd::dev::SerialTopo" in ffi.Multibody.new().jit_source(False, "rnea")
