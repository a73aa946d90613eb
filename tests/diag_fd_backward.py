"""Diagnostic (not collected by pytest): the distribution of the fp32 forward dynamics' backward
error K = |rnea64(q, qd, qdd32) - tau| / (eps32 (1 + |tau| + |H_sym| |qdd32|)) per kernel form,
over several seeds at the config-3 size, so the bound test_gpu_parity.FD32_BACKWARD_K holds is
read against the distribution's tail rather than one draw.  Test infrastructure (it runs the
oracle as the checker).  usage (GPU): python tests/diag_fd_backward.py [--seeds 4] [--batch 65536]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "rigidbody-rs_amd")]

import torch  # noqa: E402

from test_gpu_parity import fp32_fd_backward_ratio  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--batch", type=int, default=65536)
    a = ap.parse_args()
    from oracle import oracle, urdf_model
    from rigidbody_amd import chains, ffi

    xml = chains.fr3_urdf_text()
    mb = ffi.Multibody.from_urdf_string(xml)
    om = oracle.Model(urdf_model.model_raw_from_urdf(xml))
    lim = mb.limits()
    dev = torch.device("cuda:0")
    B = a.batch
    out = {}
    for form, pack in ((1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (2, 5)):
        ks = []
        worst = None
        for s in range(a.seeds):
            x = [chains.host_uniform(7, B, *chains.input_ranges(lim, k), chains.SEED + 11 + i + 100 * s,
                                     dtype="float32").astype(np.float64) for i, k in enumerate(("q", "qd", "tau"))]
            try:
                ffi.set_tuning("fd_form", form)
                ffi.set_tuning("pack", pack)
                qdd = mb.fd_batch(*[torch.as_tensor(v, dtype=torch.float32, device=dev) for v in x])
                qdd = qdd.cpu().numpy().astype(np.float64)
            finally:
                ffi.set_tuning("fd_form", -1)
                ffi.set_tuning("pack", -1)
            res = om.rnea_batch(x[0], x[1], qdd) - x[2]
            K = fp32_fd_backward_ratio(res, om.crba_batch(x[0]), qdd, x[2])
            ks.append(K.ravel())
            i = np.unravel_index(np.argmax(K), K.shape)
            if worst is None or K[i] > worst["K"]:
                worst = {"K": float(K[i]), "seed": s, "joint": int(i[0]), "col": int(i[1]),
                         "tau": float(x[2][i]), "res": float(res[i]), "qdd": float(qdd[i])}
        k = np.concatenate(ks)
        out[f"form{form}_pack{pack}"] = {"max": float(k.max()), "q99999": float(np.quantile(k, 0.99999)),
                                         "q9999": float(np.quantile(k, 0.9999)), "median": float(np.median(k)),
                                         "n": int(k.size), "worst": worst}
        print(json.dumps({f"form{form}_pack{pack}": out[f"form{form}_pack{pack}"]}), flush=True)
    print(json.dumps({"fast_trig": os.environ.get("RB_FAST_TRIG", "1"), "batch": B, "seeds": a.seeds}))


if __name__ == "__main__":
    main()
