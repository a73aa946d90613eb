"""The reference's single-configuration ABI on the host:
multibody_rnea / _crba / _fwd_kin / _jac (rigidbody_bindings/src/lib.rs:15-70) evaluate the
configuration on the calling thread with the GPU kernels' lane bodies compiled for the host
(csrc/host_eval.cpp).  CPU only: these run in the no-GPU container, against the oracle's
golden vectors (fp64, 1e-12 relative) and through the reference consumer's own calls."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, REPO, load_json, load_npz


@pytest.fixture(scope="module")
def ffi():
    from rigidbody_amd import ffi

    return ffi


def _xml(name):
    from rigidbody_amd import chains

    return chains.fr3_urdf_text() if name == "fr3" else chains.synthetic_chain_urdf(int(name[5:]))


@pytest.mark.parametrize("name", ["fr3", "chain12", "chain30"])
def test_single_config_host_matches_golden(name, ffi):
    """Every golden configuration (oracle fp64: tau, raw CRBA buffer, FK, raw Jacobian) through
    the single-configuration ABI on the host: relative 1e-12 (the oracle is the quaternion
    formulation, the lane bodies rotation matrices: a few ulp apart)."""
    mb = ffi.Multibody.from_urdf_string(_xml(name))
    assert mb.single_config_path() == "host"
    g = load_npz(f"{name}_golden.npz")
    n, B = g["q"].shape
    for b in range(B):
        q, qd, qdd = g["q"][:, b], g["qd"][:, b], g["qdd"][:, b]
        for got, want in ((mb.rnea(q, qd, qdd), g["tau"][:, b]), (mb.crba_raw(q), g["H"][:, b]),
                          (mb.fwd_kin(q), g["pos"][:, b]), (mb.jac_raw(q), g["J"][:, b])):
            assert np.abs(got - want).max() <= 1e-12 * (1 + np.abs(want).max()), (name, b)
        H = mb.crba_raw(q).reshape(n, n)  # column-major: H[col][row]
        assert np.all(H[np.triu_indices(n, 1)] == 0.0)  # strictly-lower entries exact zeros


def test_main_cpp_case_on_host(ffi):
    """The main.cpp:103-105 input (q={0,0,1,0,1,0,0}, dq={0,0,0,0,1,0,0}, ddq={1,0,0,0,0,1,0})."""
    mb = ffi.Multibody.new()
    c = load_json("main_cpp_case.json")["cases"]["main_cpp"]
    q, dq, ddq = (np.array(c[k], dtype=np.float64) for k in ("q", "dq", "ddq"))
    for got, want in ((mb.rnea(q, dq, ddq), c["tau"]), (mb.crba_raw(q), c["crba_raw"]),
                      (mb.fwd_kin(q), c["fwd_kin"]), (mb.jac_raw(q), c["jac_raw"])):
        want = np.asarray(want)
        assert np.abs(got - want).max() <= 1e-12 * (1 + np.abs(want).max())


def test_drop_in_consumer_runs_without_gpu(tmp_path):
    """examples/main_drop_in.cpp (the reference consumer's rigidbody calls) compiled against
    include/rigidbody.h, linked to librigidbody_bindings.so and run as its own process --
    config 1 end to end on a machine with no GPU."""
    exe = tmp_path / "main_drop_in"
    r = subprocess.run(["g++", "-O2", os.path.join(REPO, "examples", "main_drop_in.cpp"), "-I",
                        os.path.join(REPO, "include"), "-L", PKG, "-lrigidbody_bindings",
                        f"-Wl,-rpath,{PKG}", "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = {l.split()[0]: np.array([float(v) for v in l.split()[1:]]) for l in r.stdout.splitlines() if l}
    g = load_json("main_cpp_case.json")["cases"]["main_cpp"]
    for key, gk in (("tau", "tau"), ("pos", "fwd_kin"), ("jac", "jac_raw"), ("crba", "crba_raw")):
        want = np.asarray(g[gk])
        assert np.abs(lines[key] - want).max() <= 1e-12 * (1 + np.abs(want).max()), key


def test_single_config_argument_errors(ffi):
    """NULL inputs and handles return NULL with a message instead of aborting (the reference
    panics across FFI, lib.rs:22)."""
    import ctypes

    lib = ffi.lib()
    mb = ffi.Multibody.new()
    q = np.zeros(7)
    dp = ctypes.POINTER(ctypes.c_double)
    assert not lib.multibody_rnea(mb.handle, q.ctypes.data_as(dp), None, q.ctypes.data_as(dp))
    assert "NULL" in ffi.last_error()
    assert not lib.multibody_crba(None, q.ctypes.data_as(dp))
    assert "NULL" in ffi.last_error()


def test_single_config_path_reporting(ffi):
    """Serial revolute chains of a precompiled DOF run on the host; a tree model (hipRTC only)
    and rb_set_tuning("single_gpu", 1) report the GPU path."""
    from rigidbody_amd import chains

    assert ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30)).single_config_path() == "host"
    tree = ffi.Multibody.from_urdf_string(chains.tree_urdf(), ffi.GENERAL_AXES | ffi.URDF_TREE)
    assert tree.single_config_path() == "gpu"
    mb = ffi.Multibody.new()
    try:
        ffi.set_tuning("single_gpu", 1)
        assert mb.single_config_path() == "gpu"
    finally:
        ffi.set_tuning("single_gpu", 0)
    assert mb.single_config_path() == "host"


@pytest.mark.parametrize("n", [7, 12])
def test_general_axis_chains_on_host(n, ffi):
    """General-axis serial chains (RB_MODEL_GENERAL_AXES | RB_MODEL_URDF_TREE, SURVEY §8(f)
    rank 4) run the single-configuration ABI on the host too: the packer's per-link frame
    change plus the kTailOut rotation that fwd_kin / jac start from, against the oracle's
    general-axis reading (itself pinned to the 6x6 formulation, tests/test_general.py)."""
    from oracle import oracle, urdf_model
    from rigidbody_amd import chains

    xml = chains.general_chain_urdf(n)
    mb = ffi.Multibody.from_urdf_string(xml, ffi.URDF_TREE | ffi.GENERAL_AXES)
    assert mb.single_config_path() == "host"
    om = oracle.Model(frames=urdf_model.model_frames_from_urdf_tree(xml), general=True)
    rng = np.random.default_rng(n)
    for _ in range(8):
        q, qd, qdd = (rng.uniform(-2, 2, n) for _ in range(3))
        for got, want in ((mb.rnea(q, qd, qdd), om.rnea(q, qd, qdd)), (mb.crba_raw(q), om.crba_raw(q)),
                          (mb.fwd_kin(q), om.fwd_kin(q)), (mb.jac_raw(q), om.jac_raw(q))):
            assert np.abs(got - want).max() <= 1e-11 * (1 + np.abs(want).max()), n
