"""Operations per evaluation of the reference's own formulation, from the op-counting build of
the oracle (oracle/flops.cpp: oracle.c with `double` -> a counting type), for the workloads
bench.py reports ("pin it by an op-counting build of the CPU oracle").  CPU only;
writes profiles/r04/op_counts.json, which bench.py reads for roofline.valu.flops_per_eval_ref.

The count is data-independent except for the branch in UnitQuaternion::from_scaled_axis at
|q| ~ 0 (multibody.rs via joint.rs:48-50), so one generic configuration per model is exact for
every configuration with no zero joint angle; it is checked on a second one.

usage: python tools/op_counts.py [OUT.json]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
from oracle import oracle, urdf_model  # noqa: E402
from rigidbody_amd import chains  # noqa: E402


def counts(model, kind, n, seed):
    rng = np.random.default_rng(seed)
    q, qd, x = (rng.uniform(-1.5, 1.5, n) for _ in range(3))
    c = oracle.op_counts(model, kind, q, qd, x)
    c.pop("result")
    return c


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r04", "op_counts.json")
    res = {"method": "oracle/flops.cpp (oracle.c compiled with a counting one-double type); flops = add + mul + "
                     "div + sqrt of ONE evaluation; trig (sin / cos / acos) counted separately; the fd entry is "
                     "the A10 definition (CRBA + RNEA(q, qd, 0) + Cholesky solve)",
           "reference": "rigidbody/src/multibody.rs:41-49 (get_transforms), 111-153 (rnea), 155-174 (crba)"}
    for name, xml in (("fr3", chains.fr3_urdf_text()), ("chain30", chains.synthetic_chain_urdf(30))):
        m = oracle.Model(urdf_model.model_raw_from_urdf(xml))
        for kind in ("rnea", "crba", "fd"):
            a, b = counts(m, kind, m.n, 1), counts(m, kind, m.n, 2)
            assert a == b, (name, kind, a, b)
            res[f"{kind}_{name}"] = a
    # rollout step (aba_body.hip.hpp rollout: fd + semi-implicit Euler, qd += dt qdd; q += dt qd)
    fd = res["fd_fr3"]
    res["rollout_step_fr3"] = dict(fd, flops=fd["flops"] + 4 * 7, note="fd + 4n Euler flops")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v["flops"] for k, v in res.items() if isinstance(v, dict)}))


if __name__ == "__main__":
    main()
