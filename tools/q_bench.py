"""Time (and, under tools/profile_any.sh, profile) the q-only batched kernels of SURVEY §8(f)
ranks 1 and 3 -- multibody_crba_batch_*, multibody_jac_batch_*, multibody_fwd_kin_batch_* --
through bench.py's launcher (input sets rotated over >= 1.25 GiB, hipEvent pair around the
launches).

usage: python tools/q_bench.py --kernel crba|jac|fwd_kin [--dtype f64|f32] [--batch 1048576] [--steps 300] [--layout soa|tiled]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import bench  # noqa: E402
from rigidbody_amd import ffi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", choices=sorted(bench.Q_KERNELS), default="crba")
    ap.add_argument("--dtype", choices=["f32", "f64"], default="f64")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--layout", choices=["soa", "tiled"], default="soa")
    a = ap.parse_args()
    mb = ffi.Multibody.new()
    mb.upload()
    launch, per = bench.q_launcher(mb, a.kernel, a.batch, bench.DT[a.dtype], 1.25, layout=a.layout)
    wall, km = bench.time_launches(launch, a.steps, 5, 1, 300.0)
    print(json.dumps({"kernel": a.kernel, "dtype": a.dtype, "layout": a.layout, "batch": a.batch, "launches": a.steps,
                      "kernel_ms_avg": km, "bytes_per_eval": per // a.batch,
                      "hbm_frac": per / (km * 1e-3) / bench.HBM_PEAK,
                      "kernel_path": mb.kernel_path(a.kernel, a.dtype == "f64", a.batch)}))


if __name__ == "__main__":
    main()
