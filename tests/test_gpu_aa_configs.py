"""BASELINE.json's five configs, each at exactly its workload, against the fp64 oracle.

This file is named to be collected FIRST under `pytest -m gpu -x`, so an unrelated failure
later in the suite cannot hide a config.  Inputs are the bench's own (device splitmix64 fill,
chains.input_ranges, seed chains.SEED) on the layout bench.py times (tiled), read back to the
host for the oracle.  Reference: /root/reference/rigidbody/src/multibody.rs:111-174
(rnea, crba), rigidbody_bindings/main.cpp:66-105 (config 1's input).

Tolerances (as tests/test_gpu_parity.py):
  fp64 RNEA            |d| <= 1e-9 (1 + |tau_ref|)
  fp64 FD              torque residual |rnea64(q, qd, qdd_gpu) - tau| <= 1e-8 (1 + |tau|)
  fp32 RNEA            |d| <= 1e-4 (1 + |tau_ref|), oracle on the fp32 inputs
  fp32 FD              backward error  |r| <= 24 eps32 (1 + |tau| + |H| |qdd32|)  (FD32_BACKWARD_K)
  fp32 30-DOF RNEA     column-norm-wise 1e-4 (cancellation in the root torques, see config 5)
"""
import numpy as np
import pytest

from conftest import load_json

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ORACLE_THREADS = 16  # the GPU box's CPU share (cgroup quota)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ffi():
    from rigidbody_amd import ffi

    return ffi


def _oracle(xml):
    from oracle import oracle, urdf_model

    oracle.build()
    return oracle.Model(urdf_model.model_raw_from_urdf(xml))


def _draw(ffi, mb, kinds, B, dtype, seed):
    """The bench's inputs: one [n, B] device array per kind (bench.make_sets' fill)."""
    from rigidbody_amd import chains

    lim = mb.limits()
    out = []
    for k, kind in enumerate(kinds):
        t = torch.empty((mb.n, B), dtype=dtype, device="cuda")
        ffi.fill_uniform(t, *chains.input_ranges(lim, kind), seed + k)
        out.append(t)
    return out


def _scaled(got, ref):
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    assert np.all(np.isfinite(got)), "non-finite output"
    return float((np.abs(got - ref) / (1.0 + np.abs(ref))).max())


def _tiled(ffi, mb, kind, ins, B):
    """bench's timed path: the *_batch_tiled_* entry point on tiled copies, back to [n, B]."""
    t = [ffi.to_tiled(x) for x in ins]
    out = getattr(mb, f"{kind}_batch_tiled")(*t, B)
    return ffi.from_tiled(out, B)


# ------------------------------------------------------------------ config 1
def test_config1_single_config_main_cpp(ffi, dev):
    """Config 1: fr3 single-configuration RNEA through the reference's C ABI (multibody_new +
    multibody_rnea, lib.rs:8-30) on the main.cpp:103-105 input -- host dispatch (the default)
    and one GPU round trip per call (single_gpu) -- plus crba / fwd_kin / jac."""
    g = load_json("main_cpp_case.json")
    mb = ffi.Multibody.new()
    for single_gpu in (0, 1):
        ffi.set_tuning("single_gpu", single_gpu)
        try:
            assert mb.single_config_path() == ("gpu" if single_gpu else "host")
            for name, c in g["cases"].items():
                q, dq, ddq = (np.array(c[k], float) for k in ("q", "dq", "ddq"))
                assert _scaled(mb.rnea(q, dq, ddq), c["tau"]) <= 1e-9, name
                assert _scaled(mb.crba_raw(q), c["crba_raw"]) <= 1e-9, name
                assert _scaled(mb.fwd_kin(q), c["fwd_kin"]) <= 1e-9, name
                assert _scaled(mb.jac_raw(q), c["jac_raw"]) <= 1e-9, name
        finally:
            ffi.set_tuning("single_gpu", 0)


# ------------------------------------------------------------------ config 2
def test_config2_rnea_f32_b65536(ffi, dev, fr3_text):
    """Config 2: fr3 batched RNEA, 65536 configurations, fp32, tiled (bench's path) and SoA."""
    from rigidbody_amd import chains

    B = 65536
    mb = ffi.Multibody.new()
    q, qd, qdd = _draw(ffi, mb, ("q", "qd", "qdd"), B, torch.float32, chains.SEED)
    assert mb.kernel_path("rnea", False, B, True) == "jit"
    tau_t = _tiled(ffi, mb, "rnea", (q, qd, qdd), B).cpu().numpy()
    tau_s = mb.rnea_batch(q, qd, qdd).cpu().numpy()
    om = _oracle(fr3_text)
    h = [x.cpu().numpy().astype(np.float64) for x in (q, qd, qdd)]
    ref = om.rnea_batch(*h, nthreads=ORACLE_THREADS)
    assert _scaled(tau_t, ref) <= 1e-4
    assert _scaled(tau_s, ref) <= 1e-4


# ------------------------------------------------------------------ config 3
def test_config3_fd_f32_b65536(ffi, dev, fr3_text):
    """Config 3: fr3 batched forward dynamics, 65536 configurations, fp32 (the split packed
    waves at this size), tiled and SoA; held to the CRBA-solve definition by backward error."""
    from rigidbody_amd import chains
    from test_gpu_parity import FD32_BACKWARD_K, fp32_fd_backward_ratio

    B = 65536
    mb = ffi.Multibody.new()
    q, qd, tau = _draw(ffi, mb, ("q", "qd", "tau"), B, torch.float32, chains.SEED)
    qdd_t = _tiled(ffi, mb, "fd", (q, qd, tau), B).cpu().numpy().astype(np.float64)
    qdd_s = mb.fd_batch(q, qd, tau).cpu().numpy().astype(np.float64)
    om = _oracle(fr3_text)
    q64, qd64, t64 = (x.cpu().numpy().astype(np.float64) for x in (q, qd, tau))
    H = om.crba_batch(q64, nthreads=ORACLE_THREADS)
    for qdd32 in (qdd_t, qdd_s):
        assert np.all(np.isfinite(qdd32))
        res = om.rnea_batch(q64, qd64, qdd32, nthreads=ORACLE_THREADS) - t64
        assert fp32_fd_backward_ratio(res, H, qdd32, t64).max() <= FD32_BACKWARD_K


# ------------------------------------------------------------------ config 4
def test_config4_rnea_fd_f64(ffi, dev, fr3_text):
    """Config 4: fr3 RNEA + forward dynamics, fp64, on the global 2^20 batch and on one GPU's
    2^17 shard of it (N = 8).  The pair as bench.py times it -- multibody_rnea_fd_batch_tiled_f64,
    tau = rnea(q, qd, qdd) and qdd' = fd(q, qd, tau_in) in one launch -- against the oracle (tau
    1e-9 scaled, qdd' by its torque residual 1e-8), and the chained separate calls
    (fd(q, qd, rnea(q, qd, qdd)) = qdd, round trip).  The shard is the first 2^17 configurations
    of the 2^20 draw, launched on its own: bit for bit those columns of the full launch."""
    from rigidbody_amd import chains

    G, S = 1 << 20, 1 << 17
    mb = ffi.Multibody.new()
    assert mb.kernel_path("rnea_fd", True, G, True) == "jit" and mb.kernel_path("rnea_fd", True, S, True) == "jit"
    q, qd, qdd, tin = _draw(ffi, mb, ("q", "qd", "qdd", "tau"), G, torch.float64, chains.SEED)
    om = _oracle(fr3_text)
    h = [x.cpu().numpy() for x in (q, qd, qdd, tin)]
    t = [ffi.to_tiled(x) for x in (q, qd, qdd, tin)]
    tau_f, qdd_f = (ffi.from_tiled(o, G) for o in mb.rnea_fd_batch_tiled(*t, G))
    tau_h, qddf_h = tau_f.cpu().numpy(), qdd_f.cpu().numpy()
    assert _scaled(tau_h, om.rnea_batch(*h[:3], nthreads=ORACLE_THREADS)) <= 1e-9
    res = om.rnea_batch(h[0], h[1], qddf_h, nthreads=ORACLE_THREADS) - h[3]
    assert np.all(np.isfinite(qddf_h)) and (np.abs(res) / (1 + np.abs(h[3]))).max() <= 1e-8
    # the shard on its own
    tau_s, qdd_s = (ffi.from_tiled(o, S) for o in mb.rnea_fd_batch_tiled(*[x[: S // 256].contiguous() for x in t], S))
    assert torch.equal(tau_s, tau_f[:, :S]) and torch.equal(qdd_s, qdd_f[:, :S])
    # the separate calls, chained: fd . rnea = identity up to the conditioning of H
    tau = _tiled(ffi, mb, "rnea", (q, qd, qdd), G)
    back = _tiled(ffi, mb, "fd", (q, qd, tau), G).cpu().numpy()
    assert _scaled(back, h[2]) <= 1e-7
    assert _scaled(tau_h, tau.cpu().numpy()) <= 1e-9


# ------------------------------------------------------------------ config 5
def _normwise(got, ref):
    """Column-norm-wise scaled error max_b max_i |d_ib| / (1 + max_i |ref_ib|) (the 30-link bound:
    root torques of ~0.1 Nm left from ~3000 Nm link terms lose digits to cancellation in any fp32
    evaluation, tools/diag_c30.py; test_gpu_parity.test_chain30_full_size_f32)."""
    got, ref = np.asarray(got, float), np.asarray(ref, float)
    assert np.all(np.isfinite(got)), "non-finite output"
    return float((np.abs(got - ref).max(0) / (1 + np.abs(ref).max(0))).max())


def test_config5_chain30_rnea_f32_b1048576(ffi, dev):
    """Config 5: synthetic 30-DOF serial chain, 2^20 configurations, fp32 RNEA (the parked-force
    kernel), tiled (bench's path) and SoA: every output finite, 8193 spot columns against the
    oracle on the fp32 inputs, column-norm-wise 1e-4."""
    from rigidbody_amd import chains

    B = 1 << 20
    xml = chains.synthetic_chain_urdf(30)
    mb = ffi.Multibody.from_urdf_string(xml)
    q, qd, qdd = _draw(ffi, mb, ("q", "qd", "qdd"), B, torch.float32, chains.SEED)
    tau_t = _tiled(ffi, mb, "rnea", (q, qd, qdd), B)
    tau_s = mb.rnea_batch(q, qd, qdd)
    assert torch.isfinite(tau_t).all() and torch.isfinite(tau_s).all()
    cols = np.unique(np.concatenate([np.arange(0, B, B // 8192), [B - 1]]))
    ci = torch.as_tensor(cols, device="cuda")
    h = [x[:, ci].cpu().numpy().astype(np.float64) for x in (q, qd, qdd)]
    ref = _oracle(xml).rnea_batch(*h, nthreads=ORACLE_THREADS)
    assert _normwise(tau_t[:, ci].cpu().numpy(), ref) <= 1e-4
    assert _normwise(tau_s[:, ci].cpu().numpy(), ref) <= 1e-4
