"""The batch-size limit of one launch (capi.cpp kChunk = 2^28 configurations: lane offsets are
32-bit byte offsets, b * sizeof(T) < 2^32).  A larger batch is split into launches of at most
2^28 configurations; these tests run batches that cross that boundary with a ragged tail --
2^28 + 257 configurations, 15 GB per fp64 [7][B] array -- through the SoA and tiled entry points
and check the columns either side of the split against the oracle (fp64, 1e-9 scaled; forward
dynamics by its torque residual, 1e-8), and the tiled fp32 RNEA against the SoA one bit for bit
over the whole batch.  Reference: multibody.rs:111-174 (the algorithms), rigidbody_batch.h
(batch / ld contract)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

CHUNK = 1 << 28
B = CHUNK + 257


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if torch.cuda.get_device_properties(0).total_memory < (120 << 30):
        pytest.skip("needs > 120 GB of device memory")
    return torch.device("cuda:0")


def _fill(ffi, chains, lim, kind, dtype, seed, dev):
    """[7][B] draw within the model's ranges; the device generator takes at most 2^28 columns
    per call (rb_fill_uniform), so the columns past 2^28 come from a second seed."""
    t = torch.empty((7, B), dtype=dtype, device=dev)
    lo, hi = chains.input_ranges(lim, kind)
    ffi.fill_uniform(t[:, :CHUNK], lo, hi, seed)
    ffi.fill_uniform(t[:, CHUNK:], lo, hi, seed + 1000)
    return t


def _cols():
    rng = np.random.default_rng(5)
    return np.unique(np.r_[np.arange(64), np.arange(CHUNK - 96, CHUNK + 160), np.arange(B - 64, B),
                           rng.integers(0, B, 256)])


def test_rnea_fd_f64_across_launch_cap(dev, fr3_text):
    from oracle import oracle, urdf_model
    from rigidbody_amd import chains, ffi

    mb = ffi.Multibody.new()
    om = oracle.Model(urdf_model.model_raw_from_urdf(fr3_text))
    lim = mb.limits()
    x = {}
    for k, kind in enumerate(("q", "qd", "qdd", "tau")):
        x[kind] = _fill(ffi, chains, lim, kind, torch.float64, chains.SEED + 70 + k, dev)
    idx = torch.as_tensor(_cols(), device=dev)
    xs = {k: v[:, idx].cpu().numpy() for k, v in x.items()}
    out = torch.full((7, B), 7.0, dtype=torch.float64, device=dev)
    mb.rnea_batch(x["q"], x["qd"], x["qdd"], out=out)
    torch.cuda.synchronize()
    got = out[:, idx].cpu().numpy()
    ref = om.rnea_batch(xs["q"], xs["qd"], xs["qdd"])
    err = np.abs(got - ref) / (1 + np.abs(ref))
    assert np.isfinite(got).all() and err.max() <= 1e-9, err.max()
    del x["qdd"]
    out.fill_(7.0)
    mb.fd_batch(x["q"], x["qd"], x["tau"], out=out)
    torch.cuda.synchronize()
    qdd = out[:, idx].cpu().numpy()
    res = om.rnea_batch(xs["q"], xs["qd"], qdd) - xs["tau"]
    rr = np.abs(res) / (1 + np.abs(xs["tau"]))
    assert np.isfinite(qdd).all() and rr.max() <= 1e-8, rr.max()
    print(f"2^28 + 257 fp64: rnea {err.max():.2e}, fd residual {rr.max():.2e} over {idx.numel()} columns")


def test_rnea_f32_tiled_equals_soa_across_launch_cap(dev):
    from rigidbody_amd import chains, ffi

    mb = ffi.Multibody.new()
    lim = mb.limits()
    x = [_fill(ffi, chains, lim, kind, torch.float32, chains.SEED + 80 + k, dev)
         for k, kind in enumerate(("q", "qd", "qdd"))]
    soa = mb.rnea_batch(*x)
    tiled_in = [ffi.to_tiled(a) for a in x]
    del x
    til = mb.rnea_batch_tiled(*tiled_in, B)
    del tiled_in
    back = ffi.from_tiled(til, B)
    del til
    torch.cuda.synchronize()
    assert torch.isfinite(soa).all()
    assert torch.equal(back, soa)
