"""fp64 RNEA of serial chains longer than 8 links: the reversed-sweep kernel (rnea_body.hip.hpp
rnea_lane_rev, tuning rnea_rev, the default there) against the fp64 oracle (1e-9 scaled, every
column of small and ragged batches, spot columns at 2^20, SoA and tiled) and against the
stored-force kernel it replaces (rnea_rev = 0; the recovered kinematics add a few roundings per
link: <= 1e-11 scaled); large angles and NaN / Inf inputs as test_gpu_domain holds every other
form to.  Reference: multibody.rs:111-153."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _setup(n, general=False):
    from oracle import oracle, urdf_model
    from rigidbody_amd import chains, ffi

    if general:  # general joint axes (dense joint frames, RB_SPLIT_ROT off), as test_gpu_general
        xml = chains.general_chain_urdf(n)
        return (ffi, chains, ffi.Multibody.from_urdf_string(xml, ffi.URDF_TREE | ffi.GENERAL_AXES),
                oracle.Model(frames=urdf_model.model_frames_from_urdf_tree(xml), general=True))
    xml = chains.synthetic_chain_urdf(n)
    return ffi, chains, ffi.Multibody.from_urdf_string(xml), oracle.Model(urdf_model.model_raw_from_urdf(xml))


def _rnea(ffi, mb, x, tiled, rev):
    B = x[0].shape[1]
    try:
        ffi.set_tuning("rnea_rev", rev)
        if tiled:
            return ffi.from_tiled(mb.rnea_batch_tiled(*[ffi.to_tiled(a) for a in x], B), B)
        return mb.rnea_batch(*x)
    finally:
        ffi.set_tuning("rnea_rev", -1)


@pytest.mark.parametrize("n,general", [(12, False), (30, False), (12, True)])
def test_rev_f64_vs_oracle_and_stored_form(n, general, dev):
    ffi, chains, mb, om = _setup(n, general)
    assert mb.kernel_path("rnea", True) == "jit"
    assert "rnea_lane_rev<" in mb.jit_source(True, "rnea")
    lim = mb.limits()
    for B in (1, 63, 1000, 65536 + 77, 1 << 20):
        x = [ffi.fill_uniform(torch.empty((n, B), dtype=torch.float64, device=dev), *chains.input_ranges(lim, k),
                              chains.SEED + 90 + i) for i, k in enumerate(("q", "qd", "qdd"))]
        cols = np.arange(B) if B <= 4096 else np.unique(np.r_[np.arange(256), np.arange(B - 256, B),
                                                                np.linspace(0, B - 1, 1024).astype(int)])
        idx = torch.as_tensor(cols, device=dev)
        ref = om.rnea_batch(*[a[:, idx].cpu().numpy() for a in x])
        for tiled in (False, True):
            rev = _rnea(ffi, mb, x, tiled, -1)
            plain = _rnea(ffi, mb, x, tiled, 0)
            got = rev[:, idx].cpu().numpy()
            err = (np.abs(got - ref) / (1 + np.abs(ref))).max()
            assert np.isfinite(got).all() and err <= 1e-9, (n, B, tiled, err)
            d = ((rev - plain).abs() / (1 + plain.abs())).max().item()
            assert d <= 1e-11, (n, B, tiled, d)


def test_rev_f64_large_angles_and_nonfinite(dev):
    ffi, chains, mb, om = _setup(12)
    lim = mb.limits()
    rng = np.random.default_rng(3)
    n, B = 12, 2048 + 33
    for M in (10.0, 1e3, 1e5, 1e6):
        q = rng.choice([-1.0, 1.0], (n, B)) * M + rng.uniform(-math.pi, math.pi, (n, B))
        qd, qdd = (chains.host_uniform(n, B, *chains.input_ranges(lim, k), chains.SEED + 5 + i)
                   for i, k in enumerate(("qd", "qdd")))
        x = [torch.as_tensor(a, dtype=torch.float64, device=dev) for a in (q, qd, qdd)]
        got = _rnea(ffi, mb, x, False, -1).cpu().numpy()
        ref = om.rnea_batch(q, qd, qdd)
        err = (np.abs(got - ref) / (1 + np.abs(ref))).max()
        assert np.isfinite(got).all() and err <= 1e-9, (M, err)
    # one bad value per poisoned column, in each argument and at the root, middle and leaf joint
    x = [ffi.fill_uniform(torch.empty((n, B), dtype=torch.float64, device=dev), *chains.input_ranges(lim, k),
                          chains.SEED + 20 + i) for i, k in enumerate(("q", "qd", "qdd"))]
    clean = _rnea(ffi, mb, x, False, -1).clone()
    bad_cols = []
    for c, (a, j, v) in enumerate([(a, j, v) for a in range(3) for j in (0, 5, 11)
                                   for v in (float("nan"), float("inf"), -float("inf"))]):
        b = 7 + 40 * c
        x[a][j, b] = v
        bad_cols.append(b)
    x[0][3, 1900] = 2.0 ** 42  # an angle past the fp64 reduction range (rigidbody_batch.h)
    bad_cols.append(1900)
    out = _rnea(ffi, mb, x, False, -1)
    mask = torch.zeros(B, dtype=torch.bool, device=dev)
    mask[bad_cols] = True
    assert torch.isnan(out[:, mask]).all(), "a poisoned column has a finite torque"
    assert torch.equal(out[:, ~mask], clean[:, ~mask]), "a clean column changed"
