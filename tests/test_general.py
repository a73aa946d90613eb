"""General joint axes and the physical-tree URDF reading (behind
RB_MODEL_GENERAL_AXES / RB_MODEL_URDF_TREE) -- CPU side.

The reference has neither (z is hard-coded in its dynamics, multibody.rs:130-138, and it
pairs joints with links by index, dropping fixed joints, multibody.rs:65-77), so parity
here is pinned by two independent restatements, not by the reference:
  * oracle.c with general_axes=1 (quaternion/isometry code path) against the 6x6
    Featherstone formulation (featherstone6.py, matrices + Rodrigues) to <= 1e-11;
  * the product's C++ tree reading (model.cpp chain_from_tree) against the Python one
    (oracle/urdf_model.py model_frames_from_urdf_tree) to <= 1e-13;
and, for z-axis chains, by reduction to the reference semantics (bit-identical).
"""
import numpy as np
import pytest


def _frames(xml):
    from oracle import urdf_model

    return urdf_model.model_frames_from_urdf_tree(xml)


@pytest.mark.parametrize("n", [7, 12])
def test_general_oracle_matches_6x6(n, oracle_mod):
    from oracle import featherstone6
    from rigidbody_amd import chains

    fr = _frames(chains.general_chain_urdf(n))
    assert fr["n"] == n
    om = oracle_mod.Model(frames=fr, general=True)
    m6 = featherstone6.Model6(frames=fr, general=True)
    rng = np.random.default_rng(n)
    for _ in range(8):
        q, qd, qdd = rng.uniform(-2.5, 2.5, (3, n))
        tau = om.rnea(q, qd, qdd)
        assert np.abs(tau - m6.rnea(q, qd, qdd)).max() <= 1e-11 * (1 + np.abs(tau).max())
        H = om.crba(q)
        H6 = m6.crba(q)
        assert np.all(np.tril(H, -1) == 0.0)  # reference ABI layout kept
        assert np.abs(np.triu(H) - np.triu(H6)).max() <= 1e-12 * (1 + np.abs(H6).max())
        assert np.abs(om.jac(q) - m6.jac(q)).max() <= 1e-12
        assert np.abs(om.fwd_kin(q) - m6.fwd_kin(q)).max() <= 1e-12
        # forward dynamics: oracle definition (CRBA solve) vs ABA, and the round trip
        qdd_fd = om.fd(q, qd, tau)
        assert np.abs(qdd_fd - qdd).max() <= 1e-9 * (1 + np.abs(qdd).max())
        assert np.abs(m6.aba(q, qd, tau) - qdd).max() <= 1e-9 * (1 + np.abs(qdd).max())


def test_general_axes_reduce_to_reference_on_z_chains(oracle_mod, fr3_text):
    """With every axis +z the general motion subspace is the reference's, bit for bit."""
    from oracle import urdf_model

    raw = urdf_model.model_raw_from_urdf(fr3_text)
    ref, gen = oracle_mod.Model(raw), oracle_mod.Model(raw, general=True)
    rng = np.random.default_rng(3)
    for _ in range(16):
        q, qd, qdd = rng.uniform(-2, 2, (3, 7))
        assert np.array_equal(ref.rnea(q, qd, qdd), gen.rnea(q, qd, qdd))
        assert np.array_equal(ref.crba_raw(q), gen.crba_raw(q))
        assert np.array_equal(ref.jac_raw(q), gen.jac_raw(q))


@pytest.mark.parametrize("n", [7, 12, 30])
def test_tree_reading_cpp_matches_python(n, oracle_mod):
    from rigidbody_amd import chains, ffi

    xml = chains.general_chain_urdf(n)
    fr = _frames(xml)
    mb = ffi.Multibody.from_urdf_string(xml, ffi.GENERAL_AXES | ffi.URDF_TREE)
    assert mb.n == n and mb.flags == 3
    L = mb.blob()[5:].reshape(n, 38)
    for i in range(n):
        R = oracle_mod.quat_to_matrix(L[i, 3:7])
        assert np.abs(R - fr["Rp"][i]).max() <= 1e-13
        assert np.abs(L[i, 7:10] - fr["p"][i]).max() <= 1e-13
        assert L[i, 0:3] == pytest.approx(fr["axis"][i], abs=1e-15)
        assert L[i, 10] == pytest.approx(fr["mass"][i], rel=1e-15)
        assert np.abs(L[i, 11:14] - fr["com"][i]).max() <= 1e-13
        assert np.abs(L[i, 14:23].reshape(3, 3) - fr["icom"][i]).max() <= 1e-13
    # total moving mass: every link but world/base, fixed children included
    assert mb.total_mass == pytest.approx(fr["mass"].sum(), rel=1e-14)
    # the blob carries the flags
    mb2 = ffi.Multibody.from_blob(mb.blob())
    assert mb2.flags == 3 and np.array_equal(mb2.blob(), mb.blob(), equal_nan=True)  # continuous: NaN limits


def test_tree_reading_of_fr3_merges_the_fixed_flange(oracle_mod, fr3_text):
    """FR3 read physically: same 7 joints; fixed children merged into their parent body."""
    from oracle import urdf_model
    from rigidbody_amd import ffi

    fr = _frames(fr3_text)
    raw = urdf_model.model_raw_from_urdf(fr3_text)
    mb = ffi.Multibody.from_urdf_string(fr3_text, ffi.URDF_TREE)  # z axes: no GENERAL flag needed
    assert mb.n == fr["n"] == 7
    assert mb.total_mass == pytest.approx(fr["mass"].sum(), rel=1e-14)
    assert fr["mass"].sum() >= raw["mass"].sum() - 1e-12


def test_model_flag_errors(oracle_mod):
    from rigidbody_amd import chains, ffi

    xml = chains.general_chain_urdf(7)
    with pytest.raises(ffi.RigidBodyError, match="GENERAL_AXES"):
        ffi.Multibody.from_urdf_string(xml, ffi.URDF_TREE)
    with pytest.raises(ffi.RigidBodyError, match="flags"):
        ffi.Multibody.from_urdf_string(xml, 8)
    # branching and prismatic joints are read (tests/test_tree.py); mimic is not
    branch = xml.replace("</robot>", '  <link name="extra"/>\n  <joint name="jx" type="revolute">\n'
                         '    <parent link="body3"/>\n    <child link="extra"/>\n    <axis xyz="0 0 1"/>\n'
                         "  </joint>\n</robot>")
    mb = ffi.Multibody.from_urdf_string(branch, 3)
    par, typ = mb.topology()
    assert mb.n == 8 and list(par).count(2) == 2 and not typ.any()
    prism = xml.replace('name="j5" type="revolute"', 'name="j5" type="prismatic"')
    par, typ = ffi.Multibody.from_urdf_string(prism, 3).topology()
    assert list(par) == list(range(-1, 6)) and list(typ) == [0, 0, 0, 0, 1, 0, 0]
    mimic = xml.replace('    <child link="body4"/>', '    <child link="body4"/>\n    <mimic joint="j3"/>')
    with pytest.raises(ffi.RigidBodyError, match="mimic"):
        ffi.Multibody.from_urdf_string(mimic, 3)
    two_roots = xml.replace("</robot>", '  <link name="orphan"/>\n</robot>')
    with pytest.raises(ffi.RigidBodyError, match="root"):
        ffi.Multibody.from_urdf_string(two_roots, 3)
