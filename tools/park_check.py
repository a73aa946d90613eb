"""Bit-identity of the parked long-chain fp32 RNEA (tuning rnea_park = NP, rnea_body.hip.hpp
rnea_lane_park) against the one-per-lane kernel, 30-DOF chain, ragged and full batches, SoA and
tiled.  Needs RB_EXPERIMENTAL=1 (rnea_park is an A/B key).  Prints one JSON line."""
import json
import os
import sys

os.environ.setdefault("RB_EXPERIMENTAL", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rigidbody_amd import chains, ffi  # noqa: E402

NP = int(sys.argv[1]) if len(sys.argv) > 1 else 8
mb = ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(30))
lim = mb.limits()
res = {}
for B in (1, 63, 1000, 65539, 1 << 20):
    x = [torch.as_tensor(chains.host_uniform(30, B, *chains.input_ranges(lim, k), chains.SEED + 40 + i,
                                             dtype="float32"), device="cuda") for i, k in enumerate(("q", "qd", "qdd"))]
    out = {}
    for park in (0, NP):
        ffi.set_tuning("rnea_park", park)
        soa = mb.rnea_batch(*x).cpu().numpy()
        til = ffi.from_tiled(mb.rnea_batch_tiled(*[ffi.to_tiled(a) for a in x], B), B).cpu().numpy()
        out[park] = (soa, til)
    ffi.set_tuning("rnea_park", 0)
    res[B] = {"soa_equal": bool(np.array_equal(out[0][0], out[NP][0])),
              "tiled_equal": bool(np.array_equal(out[0][1], out[NP][1])),
              "max_abs_diff": float(np.abs(out[0][0] - out[NP][0]).max())}
print(json.dumps({"rnea_park": NP, "results": res}))
