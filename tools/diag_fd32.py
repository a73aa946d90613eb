"""Diagnostic: fp32 forward-dynamics torque residual vs the fp64 oracle per model
(run twice: RB_FAST_TRIG=1 and RB_FAST_TRIG=0)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
from oracle import oracle, urdf_model  # noqa: E402
from rigidbody_amd import chains, ffi  # noqa: E402

for name in ("fr3", "chain12", "chain30"):
    xml = chains.fr3_urdf_text() if name == "fr3" else chains.synthetic_chain_urdf(int(name[5:]))
    g = np.load(os.path.join(REPO, "tests/golden", f"{name}_golden.npz"))
    om = oracle.Model(urdf_model.model_raw_from_urdf(xml))
    mb = ffi.Multibody.from_urdf_string(xml)
    t = {k: torch.as_tensor(g[k], dtype=torch.float32, device="cuda") for k in ("q", "qd", "qdd", "tau_in")}
    q64, qd64, t64 = (g[k].astype(np.float32).astype(np.float64) for k in ("q", "qd", "tau_in"))
    qdd32 = mb.fd_batch(t["q"], t["qd"], t["tau_in"]).cpu().numpy().astype(np.float64)
    res = np.abs(om.rnea_batch(q64, qd64, qdd32) - t64) / (1 + np.abs(t64))
    ref = om.fd_batch(q64, qd64, t64)
    rel = np.abs(qdd32 - ref).max(axis=0) / (1 + np.abs(ref).max(axis=0))
    tau32 = mb.rnea_batch(t["q"], t["qd"], t["qdd"]).cpu().numpy()
    tref = om.rnea_batch(q64, qd64, g["qdd"].astype(np.float32).astype(np.float64))
    rerr = (np.abs(tau32 - tref) / (1 + np.abs(tref))).max()
    print(f"{name:8s} fast={os.environ.get('RB_FAST_TRIG', '1')} fd32 residual max {res.max():.3e} "
          f"median {np.median(res.max(axis=0)):.3e}  qdd rel max {rel.max():.3e}  rnea32 err {rerr:.3e}")
