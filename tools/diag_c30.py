"""Diagnostic: fp32 vs fp64 RNEA error on the 30-DOF chain at B = 2^20:
element-wise |d|/(1+|tau|) and column-norm-wise max|d|/(1+max|tau|) distributions; run with
RB_FAST_TRIG=1 (hardware sin/cos, default) and RB_FAST_TRIG=0."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
from rigidbody_amd import chains, ffi  # noqa: E402

for dof in (30, 7):
    mb = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(dof)) if dof != 7 else ffi.Multibody.new()
    n, B = dof, 1 << 20
    lim = mb.limits()
    x = {}
    for k, kind in enumerate(("q", "qd", "qdd")):
        lo, hi = chains.input_ranges(lim, kind)
        x[kind] = ffi.fill_uniform(torch.empty((n, B), dtype=torch.float32, device="cuda"), lo, hi, chains.SEED + k)
    t32 = mb.rnea_batch(x["q"], x["qd"], x["qdd"]).double()
    t64 = mb.rnea_batch(*(x[k].double() for k in ("q", "qd", "qdd")))
    d = (t32 - t64).abs()
    ew = d / (1 + t64.abs())
    nw = d.max(0).values / (1 + t64.abs().max(0).values)
    q = torch.tensor([0.5, 0.99, 0.9999, 1.0], device="cuda", dtype=torch.float64)
    print(f"dof {dof} fast={os.environ.get('RB_FAST_TRIG', '1')} elementwise quantiles(.5,.99,.9999,max) "
          f"{[f'{v:.2e}' for v in torch.quantile(ew.flatten()[::7], q).tolist()]} max {ew.max().item():.2e}; "
          f"normwise {[f'{v:.2e}' for v in torch.quantile(nw, q).tolist()]}; max|tau| {t64.abs().max().item():.1f}")
    j, b = divmod(int(ew.argmax()), B)
    print(f"   worst element joint {j} config {b}: tau64 {t64[j, b].item():.6g} tau32 {t32[j, b].item():.6g} "
          f"col max|tau| {t64[:, b].abs().max().item():.4g}")
