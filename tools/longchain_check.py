"""Numerics of an alternative RNEA kernel form on a synthetic long chain: the form selected by
`key=value` (RB_EXPERIMENTAL tuning, e.g. jit_variant=65536) against the default form on the same
inputs (max |d| / (1 + |tau|)), and both against the fp64 oracle on spot columns.  Diagnostic,
runs the oracle as the checker.  usage: python tools/longchain_check.py DOF key=value [f64|f32]"""
import json
import os
import sys

os.environ.setdefault("RB_EXPERIMENTAL", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rigidbody_amd import chains, ffi  # noqa: E402


def main():
    dof, kv = int(sys.argv[1]), sys.argv[2]
    dt = torch.float64 if (sys.argv[3] if len(sys.argv) > 3 else "f64") == "f64" else torch.float32
    key, val = kv.split("=")
    xml = chains.synthetic_chain_urdf(dof)
    mb = ffi.Multibody.from_urdf_string(xml)
    lim = mb.limits()
    out = {"dof": dof, "variant": kv, "dtype": str(dt)}
    for B in (1, 1000, 65536 + 77, 1 << 20):
        x = [ffi.fill_uniform(torch.empty((dof, B), dtype=dt, device="cuda"), *chains.input_ranges(lim, k),
                              chains.SEED + i) for i, k in enumerate(("q", "qd", "qdd"))]
        try:
            ffi.set_tuning(key, int(val))
            alt = mb.rnea_batch(*x).double()
        finally:
            ffi.set_tuning(key, 0 if key == "jit_variant" else -1)
        base = mb.rnea_batch(*x).double()
        rel = ((alt - base).abs() / (1 + base.abs())).max().item()
        out[f"B{B}_vs_default"] = rel
        out[f"B{B}_finite"] = bool(torch.isfinite(alt).all())
        if B == 65536 + 77:
            from oracle import oracle, urdf_model
            om = oracle.Model(urdf_model.model_raw_from_urdf(xml))
            idx = torch.linspace(0, B - 1, 512, device="cuda").long()
            xs = [v[:, idx].double().cpu().numpy() for v in x]
            ref = om.rnea_batch(*xs)
            for nm, t in (("alt", alt), ("default", base)):
                got = t[:, idx].cpu().numpy()
                out[f"oracle_{nm}"] = float((np.abs(got - ref) / (1 + np.abs(ref))).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
