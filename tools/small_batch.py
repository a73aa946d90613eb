"""Small-batch study (FR3, B = 65536): where the per-launch time
goes.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24) of

  * the no-math probe of the kernels' access pattern (probe.hip: 21 rows in / 7 out,
    tiled + non-temporal) at the same batch -- the memory-pattern + launch floor;
  * the same probe over one 256-configuration tile -- the back-to-back launch floor;
  * the RNEA / forward-dynamics kernels under each `--variants` tuning (rb_set_tuning).

usage: python tools/small_batch.py [--batch 65536] [--dtype f32] [--variants 'pack=1' 'pack=2']
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
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_lib  # noqa: E402

plib = probe_lib.lib()


def probe_launcher(B, rows_in=21, rows_out=7, nt=7):
    per = (rows_in + rows_out) * max(B, 256) * 4
    nsets = min(512, max(2, int(np.ceil(1.25 * (1 << 30) / per))))
    sets = [(torch.rand((rows_in, B), device="cuda"), torch.empty((rows_out, B), device="cuda"))
            for _ in range(nsets)]
    lib = ffi.lib()
    args = [(i.data_ptr(), o.data_ptr(), rows_in, rows_out, B, B, 1 + 16 * nt) for i, o in sets]

    def launch(i, sp):
        if plib.rb_probe_rows_f32(*args[i % nsets], sp):
            raise RuntimeError(ffi.last_error())

    launch.keep = sets
    return launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--kernels", nargs="+", default=["rnea", "fd"])
    ap.add_argument("--variants", nargs="+", default=["pack=-1"])
    a = ap.parse_args()
    dtype = bench.DT[a.dtype]
    es = 4 if a.dtype == "f32" else 8
    mb = ffi.Multibody.new()
    mb.upload()
    lib = ffi.lib()
    launches = {"probe_21x7_tiled": probe_launcher(a.batch), "probe_1tile": probe_launcher(256, 4, 4, 7)}
    for k in a.kernels:
        per = bench.set_bytes(mb.n, a.batch, es, k)
        ns = max(2, int(np.ceil(1.25 * (1 << 30) / per)))
        sets = bench.make_sets(mb, a.batch, dtype, k, ns, chains.SEED, "tiled")
        for v in a.variants:
            launches[f"{k}:{v}"] = (bench.batch_launcher(mb, sets, k, dtype, "tiled", a.batch), v)
    defaults = {"rnea_stream": -1, "grid_factor": 1, "jit": 1, "rnea_nt": -1, "fd_nt": 3, "jit_waves": -1,
                "opaque_consts": -1, "pack": -1, "f64_tab": -1, "split_rot": -1, "jit_variant": 0}
    res = {k: [] for k in launches}
    for r in range(a.rounds):
        for name, item in launches.items():
            fn, v = (item if isinstance(item, tuple) else (item, ""))
            for k, d in defaults.items():
                lib.rb_set_tuning(k.encode(), d)
            for kv in filter(None, v.split(",")):
                k, val = kv.split("=")
                assert lib.rb_set_tuning(k.encode(), int(val)) == 0, ffi.last_error()
            _, ms = bench.time_launches(fn, a.steps, 20, 1, 100.0 if r == 0 else 20.0)
            res[name].append(ms * 1e3)
    out = {}
    for name, us in res.items():
        out[name] = {"us_median": float(np.median(us)), "us_min": float(np.min(us)),
                     "us_rounds": [round(float(x), 3) for x in us]}
    print(json.dumps({"batch": a.batch, "dtype": a.dtype, "results": out}, indent=1))


if __name__ == "__main__":
    main()
