"""GPU parity for kinematic trees, prismatic joints and a floating base (SURVEY §8(f)
rank 4; RB_MODEL_URDF_TREE / RB_MODEL_FLOATING_BASE).  These models run only on the
model-specialised hipRTC kernels (tree_body.hip.hpp, the topology compiled in); the
checker is the fp64 oracle's tree form, itself pinned to the 6x6 Featherstone tree
formulation and to the free-fall invariant in tests/test_tree.py (the reference has no
trees, prismatic joints or floating base).

Tolerances as tests/test_gpu_parity.py: fp64 1e-9 * (1 + |ref|); fp32 RNEA / CRBA 1e-4;
FD through the torque residual (fp64 1e-8, fp32 1e-3).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CASES = ["tree9", "floating14"]
G = 9.81


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _setup(case):
    from oracle import oracle, urdf_model
    from rigidbody_amd import chains, ffi

    floating = case.startswith("floating")
    xml = chains.tree_urdf(floating=floating)
    flags = ffi.FLOATING_BASE if floating else ffi.URDF_TREE | ffi.GENERAL_AXES
    fr = urdf_model.model_frames_from_urdf_tree(xml, floating=floating)
    return ffi.Multibody.from_urdf_string(xml, flags), oracle.Model(frames=fr, general=True)


def _inputs(mb, B, seed):
    from rigidbody_amd import chains

    lim = mb.limits()
    rng = np.random.default_rng(seed)
    out = []
    for kind in ("q", "qd", "qdd", "tau"):
        lo, hi = (np.asarray(x, float) for x in chains.input_ranges(lim, kind))
        out.append(lo[:, None] + (hi - lo)[:, None] * rng.random((mb.n, B)))
    return out


def _t(a, dev, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=dev)


def _close(got, ref, rel, what):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    assert np.all(np.isfinite(got)), f"{what}: non-finite output"
    err = (np.abs(got - ref) / (1.0 + np.abs(ref))).max()
    assert err <= rel, f"{what}: max scaled error {err:.3e} > {rel:.1e}"


@pytest.mark.parametrize("case", CASES)
def test_tree_batched_f64(case, dev):
    from rigidbody_amd import ffi

    mb, om = _setup(case)
    n, B = mb.n, 300
    q, qd, qdd, tin = _inputs(mb, B, 5)
    for kind in ("rnea", "fd", "crba", "rollout", "fwd_kin", "jac"):
        assert mb.kernel_path(kind, True) == "jit", ffi.last_error()
    _close(mb.rnea_batch(_t(q, dev), _t(qd, dev), _t(qdd, dev)).cpu().numpy(),
           om.rnea_batch(q, qd, qdd), 1e-9, f"{case} rnea f64")
    H = mb.crba_batch(_t(q, dev)).cpu().numpy()
    _close(H, om.crba_batch(q), 1e-9, f"{case} crba f64")
    lower = np.tril(np.ones((n, n)), -1).T.reshape(-1).astype(bool)
    assert np.all(H[lower.nonzero()[0]] == 0.0)
    pos = mb.fwd_kin_batch(_t(q, dev)).cpu().numpy()
    J = mb.jac_batch(_t(q, dev)).cpu().numpy()
    for b in range(0, B, 37):
        _close(pos[:, b], om.fwd_kin(q[:, b]), 1e-9, f"{case} fwd_kin")
        _close(J[:, b], om.jac_raw(q[:, b]), 1e-9, f"{case} jac")
    qdd_gpu = mb.fd_batch(_t(q, dev), _t(qd, dev), _t(tin, dev)).cpu().numpy()
    res = om.rnea_batch(q, qd, qdd_gpu) - tin
    assert (np.abs(res) / (1 + np.abs(tin))).max() <= 1e-8, f"{case} fd f64 residual"
    _close(qdd_gpu, om.fd_batch(q, qd, tin), 1e-7, f"{case} fd f64 vs CRBA solve")
    # tiled layout: bit-identical to SoA
    tq, tqd, tqdd, ttin = (ffi.to_tiled(_t(x, dev)) for x in (q, qd, qdd, tin))
    tau_t = ffi.from_tiled(mb.rnea_batch_tiled(tq, tqd, tqdd, B), B).cpu().numpy()
    assert np.array_equal(tau_t, mb.rnea_batch(_t(q, dev), _t(qd, dev), _t(qdd, dev)).cpu().numpy())
    qdd_t = ffi.from_tiled(mb.fd_batch_tiled(tq, tqd, ttin, B), B).cpu().numpy()
    assert np.array_equal(qdd_t, qdd_gpu)
    # fp32 forward kinematics / Jacobian through the same hipRTC tree kernels -- reported as such
    # (the query resolves the kernel the launch takes, so it is built before any graph capture)
    for kind in ("fwd_kin", "jac"):
        assert mb.kernel_path(kind, False) == "jit" and mb.kernel_form(kind, False) == 1, ffi.last_error()
    q32 = _t(q, dev).float()
    q64 = q32.double().cpu().numpy()
    pos32 = mb.fwd_kin_batch(q32).cpu().numpy()
    J32 = mb.jac_batch(q32).cpu().numpy()
    for b in range(0, B, 37):
        _close(pos32[:, b], om.fwd_kin(q64[:, b]), 2e-5 * n, f"{case} fwd_kin f32")
        _close(J32[:, b], om.jac_raw(q64[:, b]), 2e-5 * n, f"{case} jac f32")


@pytest.mark.parametrize("case", CASES)
def test_tree_fd_mass_matrix_form(case, dev):
    """Forward dynamics of a tree by the mass-matrix method (fdh_body.hip.hpp fdh_eval_tree: tree
    RNEA bias + tree CRBA + L D L^T; fd_form = 2) against the oracle as the ABA is held above --
    fp64 residual 1e-8 and the CRBA solve 1e-7, fp32 residual 1e-3 norm-wise -- SoA and tiled
    bit-identical, and a NaN input poisoning exactly its own column."""
    from rigidbody_amd import ffi

    mb, om = _setup(case)
    B = 300
    q, qd, _, tin = _inputs(mb, B, 13)
    try:
        ffi.set_tuning("fd_form", 2)
        assert mb.kernel_path("fd", True) == "jit", ffi.last_error()
        qdd = mb.fd_batch(_t(q, dev), _t(qd, dev), _t(tin, dev)).cpu().numpy()
        tq, tqd, ttin = (ffi.to_tiled(_t(x, dev)) for x in (q, qd, tin))
        qdd_t = ffi.from_tiled(mb.fd_batch_tiled(tq, tqd, ttin, B), B).cpu().numpy()
        f = torch.float32
        q32, qd32, t32 = (x.astype(np.float32).astype(np.float64) for x in (q, qd, tin))
        qdd32 = mb.fd_batch(_t(q32, dev, f), _t(qd32, dev, f), _t(t32, dev, f)).cpu().numpy().astype(np.float64)
        bad = _t(tin, dev).clone()
        bad[2, 17] = float("nan")
        qdd_bad = mb.fd_batch(_t(q, dev), _t(qd, dev), bad).cpu().numpy()
    finally:
        ffi.set_tuning("fd_form", -1)
    res = om.rnea_batch(q, qd, qdd) - tin
    assert (np.abs(res) / (1 + np.abs(tin))).max() <= 1e-8, f"{case} fd f64 residual (mass-matrix form)"
    _close(qdd, om.fd_batch(q, qd, tin), 1e-7, f"{case} fd f64 vs CRBA solve (mass-matrix form)")
    assert np.array_equal(qdd_t, qdd)
    res32 = om.rnea_batch(q32, qd32, qdd32) - t32
    assert (np.abs(res32).max(axis=0) / (1 + np.abs(t32).max(axis=0))).max() <= 1e-3, f"{case} fd f32 residual"
    assert np.isnan(qdd_bad[:, 17]).all()
    keep = np.ones(B, bool)
    keep[17] = False
    assert np.array_equal(qdd_bad[:, keep], qdd[:, keep])


@pytest.mark.parametrize("case", CASES)
def test_tree_batched_f32_and_rollout(case, dev):
    mb, om = _setup(case)
    B = 256
    q, qd, qdd, tin = (x.astype(np.float32).astype(np.float64) for x in _inputs(mb, B, 9))
    f = torch.float32
    _close(mb.rnea_batch(_t(q, dev, f), _t(qd, dev, f), _t(qdd, dev, f)).cpu().numpy(),
           om.rnea_batch(q, qd, qdd), 1e-4, f"{case} rnea f32")
    _close(mb.crba_batch(_t(q, dev, f)).cpu().numpy(), om.crba_batch(q), 1e-4, f"{case} crba f32")
    qdd32 = mb.fd_batch(_t(q, dev, f), _t(qd, dev, f), _t(tin, dev, f)).cpu().numpy().astype(np.float64)
    res = om.rnea_batch(q, qd, qdd32) - tin
    assert (np.abs(res).max(axis=0) / (1 + np.abs(tin).max(axis=0))).max() <= 1e-3, f"{case} fd f32 residual"
    K, dt = 8, 1e-3
    rng = np.random.default_rng(2)
    tseq = np.stack([tin * rng.uniform(0.5, 1.0) for _ in range(K)])
    qg, qdg = _t(q, dev), _t(qd, dev)
    traj = mb.rollout_batch(qg, qdg, _t(tseq, dev), dt, traj=True)
    qK, qdK, tr = om.rollout_batch(q, qd, tseq, dt, want_traj=True)
    _close(qg.cpu().numpy(), qK, 1e-9, f"{case} rollout q")
    _close(qdg.cpu().numpy(), qdK, 1e-9, f"{case} rollout qd")
    _close(traj.cpu().numpy(), tr, 1e-9, f"{case} rollout traj")


@pytest.mark.parametrize("case", CASES)
def test_tree_single_config_abi(case, dev):
    mb, om = _setup(case)
    q, qd, qdd, _ = _inputs(mb, 4, 13)
    for b in range(4):
        _close(mb.rnea(q[:, b], qd[:, b], qdd[:, b]), om.rnea(q[:, b], qd[:, b], qdd[:, b]), 1e-9, "abi rnea")
        _close(mb.crba_raw(q[:, b]), om.crba_raw(q[:, b]), 1e-9, "abi crba")
        _close(mb.fwd_kin(q[:, b]), om.fwd_kin(q[:, b]), 1e-9, "abi fwd_kin")
        _close(mb.jac_raw(q[:, b]), om.jac_raw(q[:, b]), 1e-9, "abi jac")


def test_floating_base_free_fall_on_gpu(dev):
    mb, _ = _setup("floating14")
    n, B = mb.n, 512
    q, _, _, _ = _inputs(mb, B, 21)
    z = torch.zeros((n, B), dtype=torch.float64, device=dev)
    qdd = mb.fd_batch(_t(q, dev), z, z).cpu().numpy()
    want = np.zeros((n, 1))
    want[2] = -G
    assert np.abs(qdd - want).max() <= 1e-9
    qdd32 = mb.fd_batch(_t(q, dev, torch.float32), z.float(), z.float()).cpu().numpy()
    assert np.abs(qdd32 - want).max() <= 2e-3


def test_tree_without_jit_fails_loudly(dev):
    from rigidbody_amd import ffi

    mb, _ = _setup("tree9")
    q = torch.zeros((mb.n, 8), dtype=torch.float64, device=dev)
    try:
        ffi.set_tuning("jit", 0)
        with pytest.raises(ffi.RigidBodyError, match="hipRTC"):
            mb.rnea_batch(q, q, q)
        with pytest.raises(ffi.RigidBodyError, match="hipRTC"):
            mb.jac_batch(q)
    finally:
        ffi.set_tuning("jit", 1)
