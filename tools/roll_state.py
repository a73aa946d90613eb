"""State of the in-place fp64 / fp32 rollout after N launches of bench.rollout_launcher (the bench's
rollout line integrates one resident state launch after launch): max |q|, |qd| and the finite
fraction per launch count, so the timed region's inputs are known.  usage: python tools/roll_state.py"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import bench  # noqa: E402
from rigidbody_amd import ffi  # noqa: E402

mb = ffi.Multibody.new()
mb.upload()
for dt in (torch.float64, torch.float32):
    rl = bench.rollout_launcher(mb, 1 << 20, dt, 16)
    q, qd, _ = rl.keep
    done = 0
    for n in (0, 1, 10, 50, 100, 200, 400):
        while done < n:
            rl(done, 0)
            done += 1
        torch.cuda.synchronize()
        fin = torch.isfinite(q).all(0) & torch.isfinite(qd).all(0)
        print(json.dumps({"dtype": str(dt), "launches": n, "finite_frac": fin.double().mean().item(),
                          "q_absmax": q[:, fin].abs().max().item() if fin.any() else None,
                          "qd_absmax": qd[:, fin].abs().max().item() if fin.any() else None,
                          "q_absmed": q[:, fin].abs().median().item() if fin.any() else None}), flush=True)
