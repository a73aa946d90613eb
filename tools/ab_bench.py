"""A/B launch-shape comparison inside ONE process (interleaved rounds, median/min),
per cdna_hip_programming.md §5.4 rule 24.  Times the batched kernels over rotated
input sets (> Infinity Cache) with a hipEvent pair around `steps` launches.

usage: python tools/ab_bench.py [--kernel rnea|fd|rollout] [--dtype f32|f64] [--dof 7] [--graph]
                                [--variants 'rnea_stream=0' 'rnea_stream=1,grid_factor=2' ...]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

os.environ.setdefault("RB_EXPERIMENTAL", "1")  # A/B selectors (tuning.hpp) are experimental keys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import bench  # noqa: E402
from rigidbody_amd import chains, ffi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="rnea")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--dof", type=int, default=7)
    ap.add_argument("--model", choices=["chain", "tree9", "floating14"], default="chain",
                    help="chain: FR3 (--dof 7) or the synthetic --dof chain; tree9 / floating14: the test trees")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rollout-k", type=int, default=16, help="steps per launch for --kernel rollout")
    ap.add_argument("--layouts", nargs="+", default=["soa"], choices=["soa", "tiled"])
    ap.add_argument("--variants", nargs="+", default=["rnea_stream=0", "rnea_stream=1"],
                    help="comma-separated rb_set_tuning key=value lists; the pseudo-key 'streams' "
                         "sets how many HIP streams the timed launches rotate over")
    ap.add_argument("--graph", action="store_true",
                    help="replay the launches from a HIP graph (device-bound rate at small batches, where "
                         "eager launches from Python are host-bound)")
    a = ap.parse_args()
    dtype = bench.DT[a.dtype]
    es = 4 if a.dtype == "f32" else 8
    if a.model != "chain":
        floating = a.model == "floating14"
        mb = ffi.Multibody.from_urdf_string(chains.tree_urdf(floating=floating),
                                            ffi.FLOATING_BASE if floating else ffi.URDF_TREE | ffi.GENERAL_AXES)
    else:
        mb = ffi.Multibody.new() if a.dof == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(a.dof))
    mb.upload()
    per = bench.set_bytes(mb.n, a.batch, es, a.kernel)
    nsets = max(2, int(np.ceil(1.25 * (1 << 30) / per)))
    launches = {}
    for lay in a.layouts:
        if a.kernel == "rollout":
            launches[lay] = bench.rollout_launcher(mb, a.batch, dtype, a.rollout_k)
        elif a.kernel in bench.Q_KERNELS:  # crba / jac / fwd_kin: q in
            launches[lay] = bench.q_launcher(mb, a.kernel, a.batch, dtype, 1.25, layout=lay)[0]
        else:
            sets = bench.make_sets(mb, a.batch, dtype, a.kernel, nsets, chains.SEED, lay)
            launches[lay] = bench.batch_launcher(mb, sets, a.kernel, dtype, lay, a.batch)
    lib = ffi.lib()
    # every knob any variant sets is reset to the library default (tuning.hpp) before each
    # variant, so a knob of one variant never leaks into the next
    defaults = {"rnea_stream": -1, "grid_factor": 1, "jit": 1, "rnea_nt": -1, "fd_nt": 3, "jit_waves": -1,
                "opaque_consts": -1, "pack": -1, "f64_tab": -1, "split_rot": -1, "jit_variant": 0, "seq_tail": -1, "kin_jit": -1, "kin_nt": -1, "rnea_park": -1, "rnea_rev": -1, "kernarg_preload": 14,
                "fd_form": -1}
    used = {kv.split("=")[0] for v in a.variants for kv in v.split(",")} - {"streams"}
    keys = [(v, lp) for v in a.variants for lp in launches]
    res = {k: [] for k in keys}
    for r in range(a.rounds):
        for v, lay in keys:
            nstreams = 1
            for k in used:
                assert lib.rb_set_tuning(k.encode(), defaults[k]) == 0, ffi.last_error()
            for kv in v.split(","):
                k, val = kv.split("=")
                if k == "streams":
                    nstreams = int(val)
                    continue
                assert lib.rb_set_tuning(k.encode(), int(val)) == 0, ffi.last_error()
            print(f"round {r} variant {v} {lay}", file=sys.stderr, flush=True)
            if a.graph:  # captured per variant and round: the tuning picks the kernel at capture
                _, ms, _ = bench.time_graph(launches[lay], a.steps, spinup_ms=50.0 if r == 0 else 10.0)
            else:
                _, ms = bench.time_launches(launches[lay], a.steps, 5, 1, 50.0 if r == 0 else 0.0, nstreams)
            res[(v, lay)].append(ms)
    out = {}
    for (v, lay), ms in res.items():
        v = v + ("" if len(a.layouts) == 1 else f",{lay}")
        med = float(np.median(ms))
        out[v] = {"ms_median": med, "ms_min": float(np.min(ms)), "ms_rounds": [float(x) for x in ms],
                  "evals_per_s": a.batch / (med * 1e-3),
                  "hbm_frac": per / (med * 1e-3) / bench.HBM_PEAK}
    print(json.dumps({"kernel": a.kernel, "dtype": a.dtype, "dof": mb.n, "model": a.model, "batch": a.batch,
                      "results": out}, indent=1))


if __name__ == "__main__":
    main()
