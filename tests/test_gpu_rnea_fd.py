"""multibody_rnea_fd_batch_* (SURVEY §8(d) config 4's RNEA + forward-dynamics pair in one
launch, fdh_body.hip.hpp fdh_idfd_eval) against the oracle and against the two separate calls.

  tau     = rnea(q, qd, qdd)                    -- oracle rnea: fp64 1e-9 scaled, fp32 1e-4 scaled
                                                   on the fp32 inputs (multibody.rs:111-153)
  qdd_out = sym(H)^-1 (tau_in - rnea(q, qd, 0)) -- bit-identical to multibody_fd_batch_* (same
                                                   lane arithmetic), and in fp64 the oracle's
                                                   torque residual 1e-8 scaled (multibody.rs:155-174)

Models without the fused kernel (trees, chains over 12 links) run the RNEA then the FD kernel
inside the call: both outputs bit-identical to the separate calls there.
"""
import numpy as np
import pytest

from test_gpu_parity import _oracle, _t

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ffi():
    from rigidbody_amd import ffi

    return ffi


def _inputs(mb, B, seed, dtype=np.float64):
    from rigidbody_amd import chains

    lim = mb.limits()
    return [chains.host_uniform(mb.n, B, *chains.input_ranges(lim, k), seed + i).astype(dtype)
            for i, k in enumerate(("q", "qd", "qdd", "tau"))]


def _scaled(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    assert np.all(np.isfinite(got)), "non-finite output"
    return float((np.abs(got - ref) / (1 + np.abs(ref))).max())


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("B", [1, 255, 257, 1000, 65536 + 3, (1 << 17) + 777])
def test_rnea_fd_fr3_vs_oracle_and_separate_calls(ffi, dev, fr3_text, dt, B):
    tdt = torch.float64 if dt == "f64" else torch.float32
    mb = ffi.Multibody.new()
    assert mb.kernel_path("rnea_fd", dt == "f64", B) == "jit"
    x = _inputs(mb, B, 300 + B, np.float64 if dt == "f64" else np.float32)
    xt = [_t(a, dev, tdt) for a in x]
    tau, qdd2 = mb.rnea_fd_batch(*xt)
    # tiled: the same arithmetic on the other layout, bit for bit
    tt = [ffi.to_tiled(a) for a in xt]
    tau_t, qdd2_t = mb.rnea_fd_batch_tiled(*tt, B)
    assert torch.equal(ffi.from_tiled(tau_t, B), tau) and torch.equal(ffi.from_tiled(qdd2_t, B), qdd2)
    # qdd_out: the forward-dynamics kernel's own arithmetic
    assert torch.equal(qdd2, mb.fd_batch(xt[0], xt[1], xt[3]))
    om = _oracle(fr3_text)
    h = [a.astype(np.float64) for a in x]
    ref = om.rnea_batch(h[0], h[1], h[2], nthreads=16)
    tol = 1e-9 if dt == "f64" else 1e-4
    assert _scaled(tau.cpu().numpy(), ref) <= tol
    # against the separate RNEA kernel: the same quantity, summed in another order
    assert _scaled(tau.cpu().numpy(), mb.rnea_batch(*xt[:3]).cpu().numpy()) <= tol
    if dt == "f64":
        q2 = qdd2.cpu().numpy()
        res = om.rnea_batch(h[0], h[1], q2, nthreads=16) - h[3]
        assert (np.abs(res) / (1 + np.abs(h[3]))).max() <= 1e-8


@pytest.mark.parametrize("dt", ["f64", "f32"])
@pytest.mark.parametrize("B", [100, 65536 - 3, 1 << 17])
def test_rnea_fd_wave_split_bit_identical(ffi, dev, dt, B):
    """The wave split (pack 5, idfd_split_block1: the fp32 default up to 2^16 configurations) and
    the one-per-lane kernel (pack 1) run the same arithmetic: outputs equal bit for bit, both
    layouts; ragged batches (lanes past B store nothing)."""
    tdt = torch.float64 if dt == "f64" else torch.float32
    mb = ffi.Multibody.new()
    assert mb.kernel_form("rnea_fd", dt == "f64", B) == (5 if dt == "f32" and B <= 65536 else 1)
    x = _inputs(mb, B, 900 + B, np.float64 if dt == "f64" else np.float32)
    xt = [_t(a, dev, tdt) for a in x]
    try:
        ffi.set_tuning("pack", 5)
        assert mb.kernel_form("rnea_fd", dt == "f64", B) == 5
        split = mb.rnea_fd_batch(*xt)
        tt = [ffi.to_tiled(a) for a in xt]
        split_t = [ffi.from_tiled(o, B) for o in mb.rnea_fd_batch_tiled(*tt, B)]
        ffi.set_tuning("pack", 1)
        assert mb.kernel_form("rnea_fd", dt == "f64", B) == 1
        one = mb.rnea_fd_batch(*xt)
    finally:
        ffi.set_tuning("pack", -1)
    for a, b, c in zip(split, split_t, one):
        assert torch.equal(a, b) and torch.equal(a, c)


def test_rnea_fd_shard_of_global_batch(ffi, dev):
    """Config 4: a 2^17 shard launched on its own equals those columns of the 2^20 launch, bit
    for bit (one lane body, any grid size)."""
    from rigidbody_amd import chains

    mb = ffi.Multibody.new()
    G, S = 1 << 20, 1 << 17
    lim = mb.limits()
    xs = []
    for k, kind in enumerate(("q", "qd", "qdd", "tau")):
        t = torch.empty((7, G), dtype=torch.float64, device=dev)
        ffi.fill_uniform(t, *chains.input_ranges(lim, kind), chains.SEED + k)
        xs.append(ffi.to_tiled(t))
    tau, qdd2 = mb.rnea_fd_batch_tiled(*xs, G)
    tau_s, qdd_s = mb.rnea_fd_batch_tiled(*[x[: S // 256].contiguous() for x in xs], S)
    assert torch.equal(tau_s, tau[: S // 256]) and torch.equal(qdd_s, qdd2[: S // 256])
    assert torch.isfinite(tau).all() and torch.isfinite(qdd2).all()


@pytest.mark.parametrize("pack", [1, 5])
@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_rnea_fd_input_domain_per_output(ffi, dev, dt, pack):
    """tau is NaN exactly for configurations whose q, qd or qdd is out of the domain; qdd_out
    exactly for those whose q, qd or tau_in is (rigidbody_batch.h); neighbours untouched -- one
    per lane and the wave split (whose bias wave hands its q, qd check over in LDS)."""
    tdt = torch.float64 if dt == "f64" else torch.float32
    mb = ffi.Multibody.new()
    ffi.set_tuning("pack", pack)
    try:
        assert mb.kernel_form("rnea_fd", dt == "f64", 512) == pack
        _domain_case(ffi, mb, dev, dt, tdt)
    finally:
        ffi.set_tuning("pack", -1)


def _domain_case(ffi, mb, dev, dt, tdt):
    B = 512
    x = _inputs(mb, B, 77, np.float64 if dt == "f64" else np.float32)
    lim_angle = 2.0 ** 41 if dt == "f64" else 2.0 ** 22
    bad = {  # column -> (input index, joint, value)
        10: (0, 0, np.nan), 11: (0, 3, lim_angle * 1.5), 12: (1, 6, np.inf), 13: (2, 2, np.nan),
        14: (2, 0, -np.inf), 15: (3, 4, np.nan), 16: (3, 1, np.inf), 17: (0, 5, -lim_angle),
    }
    x[0][2, 18] = lim_angle - 4.0  # just inside the domain: finite outputs
    for c, (k, j, v) in bad.items():
        x[k][j, c] = v
    xt = [_t(a, dev, tdt) for a in x]
    tau, qdd2 = (o.cpu().numpy() for o in mb.rnea_fd_batch(*xt))
    for c in range(B):
        k = bad.get(c, (None,))[0]
        tau_bad = k in (0, 1, 2)
        fd_bad = k in (0, 1, 3)
        assert np.all(np.isnan(tau[:, c])) if tau_bad else np.all(np.isfinite(tau[:, c])), (c, "tau")
        assert np.all(np.isnan(qdd2[:, c])) if fd_bad else np.all(np.isfinite(qdd2[:, c])), (c, "qdd_out")


@pytest.mark.parametrize("model", ["chain12", "chain30", "tree9"])
def test_rnea_fd_other_models(ffi, dev, model):
    """The 12-link chain takes the fused kernel (mass-matrix forward dynamics up to 12 links);
    the 30-link chain and the tree run the RNEA then the forward-dynamics kernel inside the
    call, bit-identical to the separate calls.  tau against the separate RNEA kernel."""
    from rigidbody_amd import chains

    if model == "tree9":
        mb = ffi.Multibody.from_urdf_string(chains.tree_urdf(), ffi.URDF_TREE | ffi.GENERAL_AXES)
    else:
        mb = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(int(model[5:])))
    fused = model == "chain12"
    assert (mb.kernel_path("rnea_fd", True, 4096) == "jit") == fused
    B = 3000
    x = _inputs(mb, B, 5)
    xt = [_t(a, dev) for a in x]
    tau, qdd2 = mb.rnea_fd_batch(*xt)
    tau_ref = mb.rnea_batch(*xt[:3])
    qdd_ref = mb.fd_batch(xt[0], xt[1], xt[3])
    assert torch.equal(qdd2, qdd_ref)
    if fused:
        assert _scaled(tau.cpu().numpy(), tau_ref.cpu().numpy()) <= 1e-9
    else:
        assert torch.equal(tau, tau_ref)


@pytest.mark.parametrize("name", ["fr3_golden.npz", "chain12_golden.npz", "chain30_golden.npz"])
def test_rnea_fd_vs_golden(ffi, dev, fr3_text, name):
    """The fused pair on the committed golden vectors (tools/gen_golden.py, oracle outputs): tau
    against the golden RNEA torques at 1e-9 scaled, qdd_out against the golden CRBA-solve
    accelerations at 1e-9 cond(H)/1e3 (test_gpu_parity.test_batched_f64_vs_golden's bound)."""
    from conftest import load_npz
    from test_gpu_parity import _model_xml

    g = load_npz(name)
    mb = ffi.Multibody.from_urdf_string(_model_xml(name, fr3_text))
    n, B = g["q"].shape
    tau, qdd2 = mb.rnea_fd_batch(*[_t(g[k], dev) for k in ("q", "qd", "qdd", "tau_in")])
    assert _scaled(tau.cpu().numpy(), g["tau"]) <= 1e-9
    q2 = qdd2.cpu().numpy()
    for b in range(B):
        Hb = g["H"][:, b].reshape(n, n).T
        cond = np.linalg.cond(np.triu(Hb) + np.triu(Hb, 1).T)
        err = np.abs(q2[:, b] - g["qdd_fd"][:, b]).max() / (1 + np.abs(g["qdd_fd"][:, b]).max())
        assert err <= 1e-9 * max(1.0, cond / 1e3), (b, err, cond)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_rnea_fd_host_pointers(ffi, dev, dt):
    """multibody_rnea_fd_batch_host_*: the blocking host-pointer form equals the device form."""
    mb = ffi.Multibody.new()
    npd = np.float64 if dt == "f64" else np.float32
    x = _inputs(mb, 3001, 55, npd)
    tau_h, qdd_h = mb.rnea_fd_batch_host(*x, dtype=npd)
    assert tau_h.dtype == npd and qdd_h.dtype == npd
    tau_d, qdd_d = mb.rnea_fd_batch(*[_t(a, dev, torch.float64 if dt == "f64" else torch.float32) for a in x])
    assert np.array_equal(tau_h, tau_d.cpu().numpy()) and np.array_equal(qdd_h, qdd_d.cpu().numpy())


def test_rnea_fd_refuses_aliased_outputs(ffi, dev):
    """An output passed as an input (tau_in as tau, qdd as qdd_out) or both outputs the same
    array: RB_ERR_ARG, nothing launched (rigidbody_batch.h)."""
    mb = ffi.Multibody.new()
    x = [_t(a, dev) for a in _inputs(mb, 300, 3)]
    with pytest.raises(ffi.RigidBodyError, match="also an input"):
        mb.rnea_fd_batch(*x, tau=x[3])
    with pytest.raises(ffi.RigidBodyError, match="also an input"):
        mb.rnea_fd_batch(*x, qdd_out=x[2])
    o = torch.empty_like(x[0])
    with pytest.raises(ffi.RigidBodyError, match="same array"):
        mb.rnea_fd_batch(*x, tau=o, qdd_out=o)
