"""GPU parity over the batched ABI's whole input domain (include/rigidbody_batch.h "Input domain").

The reference evaluates any f64 joint angle exactly -- libm sin/cos inside
`UnitQuaternion::from_scaled_axis` (joint.rs:48-50, restated in oracle.c) -- and propagates NaN
/ Inf from any input through its arithmetic (multibody.rs:111-174).  These tests hold every
batched entry point and every kernel form the launch policy can pick (hipRTC and precompiled
generic; one per lane, packed pair, sequential pair, wave splits, parked long chain, ABA and
mass-matrix forward dynamics, rollouts) to the oracle there:

* large angles: q = +-M + U(-pi, pi) for M in 10 ... 1e6 rad -- and up to the supported bound,
  fp64 1e9, 1e12, 2^40 and 2^41 - 4 rad, fp32 2^22 - 4 rad -- against the oracle at the usual
  tolerances (fp64 1e-9 scaled; fp32 on the fp32-rounded inputs 1e-4 scaled for RNEA / CRBA,
  2e-5 n for fwd_kin / jac, the backward-error bound for forward dynamics -- the bounds of
  test_gpu_parity.py, unchanged);
* a continuous-joint rollout whose angles cross 100 rad, against the oracle's step-by-step
  Euler, and its 2 pi k periodicity;
* non-finite inputs: a configuration with a NaN or +-Inf anywhere among its inputs, or a joint
  angle at or beyond the supported magnitude (2^41 rad fp64, 2^22 rad fp32: exactly the bound
  and 1.5 x it), gets NaN in EVERY output
  (CRBA: every upper-triangle entry; the strictly-lower entries stay the ABI's exact zeros),
  and its neighbours -- including the other configuration of a paired lane -- are untouched.
  The reference yields NaN for every output that depends on the bad input (all of them for
  RNEA); the kernels, whose model constants fold structural zeros at compile time under
  -ffinite-math-only, guard their inputs explicitly (spatial.hip.hpp InputGuard) instead of
  relying on propagation.
"""
import math

import numpy as np
import pytest

from test_gpu_parity import FD32_BACKWARD_K, _model_xml, _oracle, _t, fp32_fd_backward_ratio

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MAGS = [10.0, 100.0, 1e3, 1e4, 1e5, 1e6]
# the batched kernels' input domain (rigidbody_batch.h, spatial.hip.hpp InputGuard): |q| < LIMIT
LIMIT = {"f64": 2.0 ** 41, "f32": 2.0 ** 22}
# magnitudes beyond MAGS up to just below the bound (M + U(-pi, pi) < LIMIT)
MAGS_HI = {"f64": [1e9, 1e12, 2.0 ** 40, 2.0 ** 41 - 4], "f32": [2.0 ** 22 - 4]}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ffi():
    from rigidbody_amd import ffi

    return ffi


# (kind, form name, tuning) -- every form the policy can take for FR3 / chains
FORMS = {
    "f64": [
        ("rnea", "auto", {}), ("rnea", "one_per_lane", {"pack": 1}), ("rnea", "generic", {"jit": 0}),
        ("rnea_tiled", "auto", {}),
        ("fd", "massmatrix", {"fd_form": 2}), ("fd", "aba", {"fd_form": 1}),
        ("fd", "split_one", {"fd_form": 2, "pack": 5}),
        ("fd", "aba_seqpair", {"fd_form": 1, "pack": 3}), ("fd", "generic", {"jit": 0}),
        ("fd_tiled", "auto", {}),
        ("crba", "auto", {}), ("crba", "generic", {"jit": 0}), ("crba_tiled", "auto", {}),
        ("fwd_kin", "auto", {}), ("fwd_kin", "generic", {"jit": 0}),
        ("jac", "auto", {}), ("jac", "generic", {"jit": 0}), ("jac_tiled", "auto", {}),
    ],
    "f32": [
        ("rnea", "auto", {}), ("rnea", "seqpair", {"pack": 3}), ("rnea", "generic", {"jit": 0}),
        ("rnea_tiled", "auto", {}),
        ("fd", "massmatrix", {"fd_form": 2, "pack": 1}), ("fd", "massmatrix_pair", {"fd_form": 2, "pack": 2}),
        ("fd", "split_packed", {"fd_form": 2, "pack": 4}), ("fd", "split_one", {"fd_form": 2, "pack": 5}),
        ("fd", "aba", {"fd_form": 1, "pack": 1}), ("fd", "aba_pair", {"fd_form": 1, "pack": 2}),
        ("fd", "generic", {"jit": 0}), ("fd_tiled", "auto", {}),
        ("crba", "auto", {}), ("crba", "generic", {"jit": 0}),
        ("fwd_kin", "auto", {}), ("fwd_kin", "generic", {"jit": 0}),
        ("jac", "auto", {}), ("jac", "generic", {"jit": 0}),
    ],
}
DEFAULTS = {"jit": 1, "pack": -1, "fd_form": -1, "rnea_park": -1}


def _tuned(ffi, tuning, fn):
    try:
        for k, v in tuning.items():
            ffi.set_tuning(k, v)
        return fn()
    finally:
        for k in tuning:
            ffi.set_tuning(k, DEFAULTS[k])


def _run(ffi, mb, kind, x, dtype, tuning):
    """Output of one batched entry point as a float64 numpy array [rows, B]."""
    B = x["q"].shape[1]
    t = x

    def call():
        base = kind.replace("_tiled", "")
        args = {"rnea": ("q", "qd", "qdd"), "fd": ("q", "qd", "tau"), "crba": ("q",), "fwd_kin": ("q",),
                "jac": ("q",)}[base]
        if kind.endswith("_tiled"):
            out = getattr(mb, f"{base}_batch_tiled")(*[ffi.to_tiled(t[a]) for a in args], B)
            return ffi.from_tiled(out, B)
        return getattr(mb, f"{base}_batch")(*[t[a] for a in args])

    out = _tuned(ffi, tuning, call)
    return out.cpu().numpy().astype(np.float64)


def _inputs(n, B, M, seed, lim, dtype):
    from rigidbody_amd import chains

    rng = np.random.default_rng(seed)
    q = rng.choice([-1.0, 1.0], (n, B)) * M + rng.uniform(-math.pi, math.pi, (n, B))
    x = {"q": q}
    for i, k in enumerate(("qd", "qdd", "tau")):
        x[k] = chains.host_uniform(n, B, *chains.input_ranges(lim, k), chains.SEED + 300 + i)
    np_dt = np.float32 if dtype == torch.float32 else np.float64
    return {k: v.astype(np_dt).astype(np.float64) for k, v in x.items()}


def _check(kind, got, x, om, dt, n):
    """Max error of one output against the oracle, normalised so <= 1 passes."""
    base = kind.replace("_tiled", "")
    f64 = dt == "f64"
    if not np.all(np.isfinite(got)):
        return np.inf
    if base == "rnea":
        ref = om.rnea_batch(x["q"], x["qd"], x["qdd"])
        return (np.abs(got - ref) / (1 + np.abs(ref))).max() / (1e-9 if f64 else 1e-4)
    if base == "crba":
        ref = om.crba_batch(x["q"])
        return (np.abs(got - ref) / (1 + np.abs(ref))).max() / (1e-9 if f64 else 1e-4)
    if base in ("fwd_kin", "jac"):
        B = x["q"].shape[1]
        cols = range(0, B, max(1, B // 128))
        f = om.fwd_kin if base == "fwd_kin" else om.jac_raw
        err = max((np.abs(got[:, b] - f(x["q"][:, b])) / (1 + np.abs(f(x["q"][:, b])))).max() for b in cols)
        return err / (1e-9 if f64 else 2e-5 * n)
    # forward dynamics: torque residual and, fp32, the backward-error bound (test_gpu_parity)
    res = om.rnea_batch(x["q"], x["qd"], got) - x["tau"]
    if f64:
        return (np.abs(res) / (1 + np.abs(x["tau"]))).max() / 1e-8
    r1 = (np.abs(res) / (1 + np.abs(x["tau"]))).max() / 1e-3
    r2 = fp32_fd_backward_ratio(res, om.crba_batch(x["q"]), got, x["tau"]).max() / FD32_BACKWARD_K
    return max(r1, r2)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_large_angles_every_form(dt, ffi, dev, fr3_text):
    """FR3, every entry point and kernel form, |q| ~ 10 ... 1e6 rad and up to just below the
    supported bound (MAGS_HI), against the oracle."""
    mb = ffi.Multibody.from_urdf_string(fr3_text)
    om = _oracle(fr3_text)
    lim = mb.limits()
    dtype = torch.float64 if dt == "f64" else torch.float32
    bad = []
    worst = {}
    for mi, M in enumerate(MAGS + MAGS_HI[dt]):
        x = _inputs(7, 2048 + 77, M, 1000 + mi, lim, dtype)
        assert np.abs(x["q"]).max() < LIMIT[dt]
        xt = {k: _t(v, dev, dtype) for k, v in x.items()}
        for kind, form, tuning in FORMS[dt]:
            got = _run(ffi, mb, kind, xt, dtype, tuning)
            r = _check(kind, got, x, om, dt, 7)
            worst[(kind, form)] = max(worst.get((kind, form), 0.0), r)
            if not r <= 1.0:
                bad.append(f"{kind}/{form} M={M:g}: {r:.3g}x tolerance")
    print({f"{k}/{f}": round(v, 4) for (k, f), v in worst.items()})
    assert not bad, "\n".join(bad)


def test_large_angles_long_chain_f32(ffi, dev):
    """The 30-DOF chain's fp32 RNEA (parked-force form, the config-5 kernel, and unparked) and
    forward dynamics (ABA) at large angles."""
    from rigidbody_amd import chains

    xml = chains.synthetic_chain_urdf(30)
    mb = ffi.Multibody.from_urdf_string(xml)
    om = _oracle(xml)
    lim = mb.limits()
    bad = []
    for mi, M in enumerate(MAGS):
        x = _inputs(30, 1024 + 5, M, 2000 + mi, lim, torch.float32)
        xt = {k: _t(v, dev, torch.float32) for k, v in x.items()}
        for kind, form, tuning in (("rnea", "parked", {}), ("rnea", "unparked", {"rnea_park": 0}),
                                   ("rnea", "generic", {"jit": 0})):
            got = _run(ffi, mb, kind, xt, torch.float32, tuning)
            ref = om.rnea_batch(x["q"], x["qd"], x["qdd"])
            # column-norm-wise, as test_chain30_full_size_f32 (cancellation in the root torques)
            r = (np.abs(got - ref).max(0) / (1 + np.abs(ref).max(0))).max() / 1e-4
            if not r <= 1.0:
                bad.append(f"{kind}/{form} M={M:g}: {r:.3g}x tolerance")
        got = _run(ffi, mb, "fd", xt, torch.float32, {})
        res = om.rnea_batch(x["q"], x["qd"], got) - x["tau"]
        r = fp32_fd_backward_ratio(res, om.crba_batch(x["q"]), got, x["tau"]).max() / FD32_BACKWARD_K
        if not r <= 1.0:
            bad.append(f"fd M={M:g}: {r:.3g}x tolerance")
    assert not bad, "\n".join(bad)


def test_large_angles_single_config_abi(ffi, dev, fr3_text):
    """multibody_rnea / _crba / _fwd_kin / _jac (lib.rs:15-70) at any finite angle, up to 1e15
    rad: the host path falls back to libm past the kernels' reduction range, as the reference."""
    mb = ffi.Multibody.new()
    om = _oracle(fr3_text)
    rng = np.random.default_rng(7)
    for M in MAGS + [1e9, 1e12, 2.0 ** 46, 1e15]:
        for _ in range(8):
            q = rng.choice([-1.0, 1.0], 7) * M + rng.uniform(-math.pi, math.pi, 7)
            qd, qdd = rng.uniform(-2, 2, 7), rng.uniform(-10, 10, 7)
            for got, ref, what in ((mb.rnea(q, qd, qdd), om.rnea(q, qd, qdd), "rnea"),
                                   (mb.crba_raw(q), om.crba_raw(q), "crba"),
                                   (mb.fwd_kin(q), om.fwd_kin(q), "fwd_kin"),
                                   (mb.jac_raw(q), om.jac_raw(q), "jac")):
                err = (np.abs(got - ref) / (1 + np.abs(ref))).max()
                assert err <= 1e-9, (what, M, err)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_rollout_continuous_joints_past_100_rad(dt, ffi, dev, fr3_text):
    """A rollout whose joints turn through 100 rad (the 7 joints as continuous: angles start at
    +-(99.5-99.9) rad and move outwards at 3-5 rad/s for 128 steps of 1 ms), every rollout form,
    against the oracle's step-by-step semi-implicit Euler on the same (fp32-rounded) start; fp64
    also against the same rollout started 2 pi * 15 closer to 0, which must agree up to that
    offset (the dynamics are 2 pi-periodic in every revolute angle)."""
    mb = ffi.Multibody.from_urdf_string(fr3_text)
    om = _oracle(fr3_text)
    dtype = torch.float64 if dt == "f64" else torch.float32
    npd = np.float64 if dt == "f64" else np.float32
    K, step, B = 128, 1e-3, 1024 + 3
    rng = np.random.default_rng(11)
    sign = rng.choice([-1.0, 1.0], (7, B))
    q0 = (sign * rng.uniform(99.5, 99.9, (7, B))).astype(npd).astype(np.float64)
    qd0 = (sign * rng.uniform(3.0, 5.0, (7, B))).astype(npd).astype(np.float64)
    tau = (rng.uniform(-5, 5, (K, 7, B))).astype(npd).astype(np.float64)
    qr, qdr, tr = om.rollout_batch(q0, qd0, tau, step, want_traj=True)
    assert np.abs(tr).max() > 100.0 and np.abs(q0).max() < 100.0
    tol = 1e-9 if dt == "f64" else 1e-4
    for form, tuning in (("auto", {}), ("pair", {"pack": 2}), ("one_per_lane", {"pack": 1}),
                         ("aba", {"fd_form": 1}), ("generic", {"jit": 0})):
        q, qd = _t(q0, dev, dtype), _t(qd0, dev, dtype)
        ts = torch.as_tensor(tau, dtype=dtype, device=dev).contiguous()
        traj = _tuned(ffi, tuning, lambda: mb.rollout_batch(q, qd, ts, step, traj=True)).cpu().numpy()
        # scaled per step by the trajectory's own magnitude (|q| ~ 100: fp32 ulp 7.6e-6)
        err = (np.abs(traj - tr) / (1 + np.abs(tr))).max()
        assert np.all(np.isfinite(traj)) and err <= tol * 10, (dt, form, err)
        errv = (np.abs(qd.cpu().numpy() - qdr) / (1 + np.abs(qdr))).max()
        assert errv <= tol * 100, (dt, form, "qd", errv)
        if dt == "f64" and form == "auto":
            off = sign * (2 * math.pi * 15)
            q1, qd1 = _t(q0 - off, dev, dtype), _t(qd0, dev, dtype)
            traj1 = mb.rollout_batch(q1, qd1, ts, step, traj=True).cpu().numpy()
            np.testing.assert_allclose(traj1 + off[None], traj, rtol=0, atol=1e-9)
            np.testing.assert_allclose(qd1.cpu().numpy(), qd.cpu().numpy(), rtol=1e-9, atol=1e-9)


# ---------------------------------------------------------------- non-finite inputs
def _poisoned(n, B, lim, dt, args, seed, poison=None, boundary=True):
    """Inputs with one bad value per poisoned column: for each argument, joint and value in
    (NaN, +Inf, -Inf, and for q +-1.5 x the supported magnitude and, with `boundary`, +-exactly
    that magnitude), one column.  Returns the
    inputs and the poisoned column indices (all in the first 256-column block, so every
    paired-lane partner in the next block is clean)."""
    from rigidbody_amd import chains

    x = {}
    for i, k in enumerate(args):
        x[k] = chains.host_uniform(n, B, *chains.input_ranges(lim, k), seed + i)
    cols = []
    c = 0
    for k in poison or args:
        vals = [np.nan, np.inf, -np.inf] + ([1.5 * LIMIT[dt], -1.5 * LIMIT[dt]] if k == "q" else []) + \
               ([LIMIT[dt], -LIMIT[dt]] if k == "q" and boundary else [])
        for j in range(n):
            for v in vals:
                x[k][j, c] = v
                cols.append(c)
                c += 1
    assert c <= 256
    np_dt = np.float32 if dt == "f32" else np.float64
    return {k: v.astype(np_dt).astype(np.float64) for k, v in x.items()}, np.array(cols)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_nonfinite_inputs_every_form(dt, ffi, dev, fr3_text):
    """NaN / +-Inf / out-of-range angles in any input of a configuration: every output of that
    configuration is NaN (CRBA: the upper triangle; the lower stays exactly 0), in every
    kernel form; every clean configuration -- including the other half of a paired lane and
    of a sequential pair -- still matches the oracle."""
    mb = ffi.Multibody.from_urdf_string(fr3_text)
    om = _oracle(fr3_text)
    lim = mb.limits()
    dtype = torch.float64 if dt == "f64" else torch.float32
    n, B = 7, 1024 + 17
    lower = np.tril(np.ones((n, n)), -1).T.reshape(-1).astype(bool)  # column-major strictly lower
    bad = []
    for kind, form, tuning in FORMS[dt]:
        base = kind.replace("_tiled", "")
        args = {"rnea": ("q", "qd", "qdd"), "fd": ("q", "qd", "tau")}.get(base, ("q",))
        x, cols = _poisoned(n, B, lim, dt, args, 4000)
        xt = {k: _t(v, dev, dtype) for k, v in x.items()}
        got = _run(ffi, mb, kind, xt, dtype, tuning)
        rows = ~lower if base == "crba" else np.ones(got.shape[0], bool)
        nf = ~np.isfinite(got[np.ix_(rows, cols)])
        if not nf.all():
            miss = cols[~nf.all(0)]
            bad.append(f"{kind}/{form}: {len(miss)} poisoned columns with finite outputs, e.g. {miss[:6].tolist()}")
        if base == "crba" and not np.all(got[np.ix_(lower, cols)] == 0.0):
            bad.append(f"{kind}/{form}: lower triangle of a poisoned column not exactly 0")
        clean = np.setdiff1d(np.arange(B), cols)
        xc = {k: v[:, clean] for k, v in x.items()}
        r = _check(kind, got[:, clean], xc, om, dt, n)
        if not r <= 1.0:
            bad.append(f"{kind}/{form}: clean columns {r:.3g}x tolerance")
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("dt", ["f64", "f32"])
def test_nonfinite_long_chain_and_rollout(dt, ffi, dev, fr3_text):
    """The same rule for the 30-DOF chain's RNEA (parked and unparked; fp32 and fp64) and for
    rollouts: a NaN / Inf in the start state poisons the whole trajectory of that configuration;
    one in tau at step k poisons its trajectory from step k on (the steps before stay the
    oracle's), every form."""
    from rigidbody_amd import chains

    dtype = torch.float64 if dt == "f64" else torch.float32
    xml = chains.synthetic_chain_urdf(30)
    mb30 = ffi.Multibody.from_urdf_string(xml)
    om30 = _oracle(xml)
    # 30 joints x 8 values: the q and qd columns fill the first block
    x, cols = _poisoned(30, 1000, mb30.limits(), dt, ("q", "qd", "qdd"), 5000, poison=("q", "qd"), boundary=False)
    bad = []
    xt = {k: _t(v, dev, dtype) for k, v in x.items()}
    for form, tuning in (("auto", {}), ("unparked", {"rnea_park": 0})):
        got = _run(ffi, mb30, "rnea", xt, dtype, tuning)
        poisoned = ~(np.isfinite(x["q"]) & (np.abs(x["q"]) < LIMIT[dt])).all(0) | ~np.isfinite(x["qd"]).all(0)
        pc = np.nonzero(poisoned)[0]
        if not (~np.isfinite(got[:, pc])).all():
            bad.append(f"chain30 rnea/{form}: poisoned columns with finite outputs")
        clean = np.nonzero(~poisoned)[0]
        ref = om30.rnea_batch(*[x[k][:, clean] for k in ("q", "qd", "qdd")])
        tol = 1e-9 if dt == "f64" else 1e-4
        r = (np.abs(got[:, clean] - ref).max(0) / (1 + np.abs(ref).max(0))).max()
        if not r <= tol:
            bad.append(f"chain30 rnea/{form}: clean columns {r:.3g}")
    # rollouts, FR3
    mb = ffi.Multibody.from_urdf_string(fr3_text)
    om = _oracle(fr3_text)
    K, step, B = 12, 1e-3, 700
    rng = np.random.default_rng(13)
    npd = np.float64 if dt == "f64" else np.float32
    q0 = rng.uniform(-2, 2, (7, B)).astype(npd).astype(np.float64)
    qd0 = rng.uniform(-1, 1, (7, B)).astype(npd).astype(np.float64)
    tau = rng.uniform(-5, 5, (K, 7, B)).astype(npd).astype(np.float64)
    first_bad = np.full(B, K)  # step from which a column's trajectory must be NaN
    c = 0
    for arr in ("q", "qd"):
        for j in range(7):
            (q0 if arr == "q" else qd0)[j, c] = [np.nan, np.inf, -np.inf][c % 3]
            first_bad[c] = 0
            c += 1
    for k in (0, 5, 11):
        for j in (0, 3, 6):
            tau[k, j, c] = [np.nan, np.inf, -np.inf][c % 3]
            first_bad[c] = k
            c += 1
    clean = first_bad == K
    qr, qdr, tr = om.rollout_batch(q0[:, clean], qd0[:, clean], tau[:, :, clean], step, want_traj=True)
    for form, tuning in (("auto", {}), ("pair", {"pack": 2}), ("one_per_lane", {"pack": 1}),
                         ("aba", {"fd_form": 1}), ("generic", {"jit": 0})):
        q, qd = _t(q0, dev, dtype), _t(qd0, dev, dtype)
        ts = torch.as_tensor(tau, dtype=dtype, device=dev).contiguous()
        traj = _tuned(ffi, tuning, lambda: mb.rollout_batch(q, qd, ts, step, traj=True)).cpu().numpy()
        for b in np.nonzero(~clean)[0]:
            k = first_bad[b]
            if not (~np.isfinite(traj[k:, :, b])).all():
                bad.append(f"rollout/{form}: column {b} finite after its bad input at step {k}")
                break
            if k > 0 and not np.isfinite(traj[:k, :, b]).all():
                bad.append(f"rollout/{form}: column {b} non-finite before step {k}")
                break
        if not (~np.isfinite(q.cpu().numpy()[:, ~clean])).all():
            bad.append(f"rollout/{form}: final q of a poisoned column finite")
        tol = 1e-9 if dt == "f64" else 1e-4
        err = (np.abs(traj[:, :, clean] - tr) / (1 + np.abs(tr))).max()
        if not err <= tol:
            bad.append(f"rollout/{form}: clean columns {err:.3g}")
    assert not bad, "\n".join(bad)


def test_nonfinite_single_config_abi(ffi, dev, fr3_text):
    """The single-configuration ABI (host path and the GPU launch of single_gpu = 1): a NaN / Inf
    input gives NaN in every output, as the reference's RNEA does for every torque."""
    mb = ffi.Multibody.new()
    rng = np.random.default_rng(9)
    q0, qd0, qdd0 = (rng.uniform(-1, 1, 7) for _ in range(3))
    try:
        for single_gpu in (0, 1):
            ffi.set_tuning("single_gpu", single_gpu)
            for arr in ("q", "qd", "qdd"):
                for j in range(7):
                    for v in (np.nan, np.inf, -np.inf):
                        x = {"q": q0.copy(), "qd": qd0.copy(), "qdd": qdd0.copy()}
                        x[arr][j] = v
                        tau = mb.rnea(x["q"], x["qd"], x["qdd"])
                        assert (~np.isfinite(tau)).all(), (single_gpu, arr, j, v, tau)
                        if arr == "q":
                            H = mb.crba_raw(x["q"])
                            up = ~np.tril(np.ones((7, 7)), -1).T.reshape(-1).astype(bool)
                            assert (~np.isfinite(H[up])).all() and np.all(H[~up] == 0.0), (single_gpu, j, v)
                            assert (~np.isfinite(mb.fwd_kin(x["q"]))).all(), (single_gpu, j, v)
                            assert (~np.isfinite(mb.jac_raw(x["q"]))).all(), (single_gpu, j, v)
    finally:
        ffi.set_tuning("single_gpu", 0)


@pytest.mark.parametrize("case", ["tree9", "floating14"])
def test_trees_domain(case, dev):
    """Kinematic trees / a floating base (tree_body.hip.hpp): revolute angles
    moved by +-159 turns (|q| ~ 1e3) against the oracle's tree form (prismatic coordinates stay in their ranges -- a
    displacement is not reduced), and NaN / Inf in any input of a configuration giving NaN in every
    output of RNEA, forward dynamics, CRBA (upper triangle), fwd_kin and jac, fp64 and fp32."""
    import test_gpu_tree as tt

    mb, om = tt._setup(case)
    n = mb.n
    _, typ = mb.topology()
    rev = typ == 0
    B = 600
    q, qd, qdd, tau = tt._inputs(mb, B, 77)
    rng = np.random.default_rng(78)
    # +-159 turns (~1e3 rad): the configuration, and so the conditioning of H (the floating base's
    # pitch joint is singular at +-pi/2), stays the in-range one
    q[rev] += rng.choice([-1.0, 1.0], (int(rev.sum()), B)) * (2 * math.pi * 159)
    for dtype, tol in ((torch.float64, 1e-9), (torch.float32, 1e-4)):
        npd = np.float64 if dtype == torch.float64 else np.float32
        x = [a.astype(npd).astype(np.float64) for a in (q, qd, qdd, tau)]
        t = [tt._t(a, dev, dtype) for a in x]
        tau_g = mb.rnea_batch(t[0], t[1], t[2]).cpu().numpy().astype(np.float64)
        ref = om.rnea_batch(x[0], x[1], x[2])
        err = (np.abs(tau_g - ref).max(0) / (1 + np.abs(ref).max(0))).max()
        assert err <= tol, (case, dtype, "rnea", err)
        H = mb.crba_batch(t[0]).cpu().numpy().astype(np.float64)
        errh = (np.abs(H - om.crba_batch(x[0])) / (1 + np.abs(om.crba_batch(x[0])))).max()
        assert errh <= tol, (case, dtype, "crba", errh)
        qdd_g = mb.fd_batch(t[0], t[1], t[3]).cpu().numpy().astype(np.float64)
        res = om.rnea_batch(x[0], x[1], qdd_g) - x[3]
        assert (np.abs(res) / (1 + np.abs(x[3]))).max() <= (1e-8 if dtype == torch.float64 else 1e-3), (case, dtype)
        # non-finite inputs, one per column, every argument and joint
        xp = [a.copy() for a in x]
        cols = []
        c = 0
        for a in (0, 1, 2, 3):
            for j in range(n):
                xp[a][j, c] = [np.nan, np.inf, -np.inf][c % 3]
                cols.append((a, c))
                c += 1
        tp = [tt._t(a, dev, dtype) for a in xp]
        outs = {"rnea": (mb.rnea_batch(tp[0], tp[1], tp[2]), (0, 1, 2)),
                "fd": (mb.fd_batch(tp[0], tp[1], tp[3]), (0, 1, 3)),
                "crba": (mb.crba_batch(tp[0]), (0,)), "fwd_kin": (mb.fwd_kin_batch(tp[0]), (0,)),
                "jac": (mb.jac_batch(tp[0]), (0,))}
        upper = ~np.tril(np.ones((n, n)), -1).T.reshape(-1).astype(bool)
        for name, (o, args) in outs.items():
            o = o.cpu().numpy()
            rows = upper if name == "crba" else np.ones(o.shape[0], bool)
            for a, col in cols:
                if a in args:
                    assert (~np.isfinite(o[rows, col])).all(), (case, dtype, name, a, col)
            clean = [col for col in range(c, B)]
            assert np.isfinite(o[:, clean]).all(), (case, dtype, name)


# ---------------------------------------------------------------- near-singular H, fp64
# The fp64 forward dynamics near a singular mass matrix, judged by the bounds of a backward-stable
# solve (L D L^T / Cholesky of an SPD matrix is normwise backward stable) rather than by a fixed
# torque residual (rigidbody_batch.h "Accuracy"), with H_s = sym(H) and C = rnea(q, qd, 0) from
# the oracle (multibody.rs:155-174 and :111-153 at qdd = 0):
#   backward:  |H_s qdd - (tau - C)|_inf <= FD64_BACKWARD_K n eps64 (|H_s|_inf |qdd|_inf + |tau - C|_inf)
#   forward:   |qdd - qdd_oracle|_inf <= FD64_FORWARD_K eps64 cond(H_s) (1 + |qdd_oracle|_inf)
# (qdd_oracle: the oracle's fp64 Cholesky solve; its own backward ratio on this draw is 0.26 / n; the
# kernels measured 0.03-0.04 backward, 0.19-0.23 forward, profiles/r06/session3/tests.log).
# The torque residual through the RNEA is no judge here: at pitch -> +-pi/2 the solution grows
# like cond(H) and the RNEA's own rounding of the cancelling link accelerations exceeds the fixed
# 1e-8 (round 5: 1.08e-7 at ~1e3 rad offsets; the oracle's own solve fails it too).
FD64_BACKWARD_K = 1.0
FD64_FORWARD_K = 4.0


def test_fd64_near_singular_floating_base(dev):
    """The floating base's mass matrix is singular at pitch = +-pi/2 (the virtual joints' Euler
    angles, rigidbody_batch.h RB_MODEL_FLOATING_BASE).  Pitch within 1e-3 ... 1e-6 of +-pi/2
    (cond(H) 6e7 ... 1e14), every fp64 forward-dynamics form of the tree (the ABA default and the
    mass-matrix form), against the two bounds above; the last quarter of the batch is the ordinary
    draw (cond(H) < 1e4), held to the usual 1e-8 torque residual as well."""
    import test_gpu_tree as tt
    from rigidbody_amd import ffi

    mb, om = tt._setup("floating14")
    n = mb.n
    B = 1024
    q, qd, _, tau = tt._inputs(mb, B, 91)
    rng = np.random.default_rng(92)
    delta = 10.0 ** rng.uniform(-6, -3, B)
    near = np.arange(B) < 3 * B // 4
    q[4, near] = (rng.choice([-1.0, 1.0], B) * (math.pi / 2 - delta))[near]
    H = om.crba_batch(q)
    Hm = H.reshape(n, n, B).transpose(2, 1, 0)  # [b, row, col], upper triangle
    Hs = np.triu(Hm) + np.triu(Hm, 1).transpose(0, 2, 1)
    cond = np.linalg.cond(Hs)
    assert cond[near].max() > 1e12 and cond[~near].max() < 1e4, (cond[near].max(), cond[~near].max())
    ref = om.fd_batch(q, qd, tau)
    y = tau - om.rnea_batch(q, qd, np.zeros_like(q))
    eps = float(np.finfo(np.float64).eps)
    normH = np.abs(Hs).sum(2).max(1)
    worst = {}
    for form, tuning in (("aba", {}), ("massmatrix", {"fd_form": 2})):
        got = _tuned(ffi, tuning, lambda: mb.fd_batch(_t(q, dev), _t(qd, dev), _t(tau, dev))).cpu().numpy()
        assert np.isfinite(got).all(), form
        r = np.einsum("brc,cb->rb", Hs, got) - y
        kb = (np.abs(r).max(0) / (n * eps * (normH * np.abs(got).max(0) + np.abs(y).max(0)))).max()
        kf = (np.abs(got - ref).max(0) / (eps * cond * (1 + np.abs(ref).max(0)))).max()
        res = om.rnea_batch(q[:, ~near], qd[:, ~near], got[:, ~near]) - tau[:, ~near]
        worst[form] = (kb, kf)
        assert kb <= FD64_BACKWARD_K, (form, "backward", kb)
        assert kf <= FD64_FORWARD_K, (form, "forward", kf)
        assert (np.abs(res) / (1 + np.abs(tau[:, ~near]))).max() <= 1e-8, form
    print("near-singular floating base fp64 FD, (backward K, forward K):", worst, f"cond(H) max {cond.max():.2e}")
