"""Sustained-load drift of per-launch time: the headline RNEA launch vs the no-math probe of
the same access pattern (tiled, non-temporal; probe.hip), each run back-to-back for a few
thousand launches over rotated buffers, timed per chunk of 100 launches (one hipEvent pair
per chunk).  Separates clock/power behaviour of the memory system (both drift) from
behaviour tied to the kernel's own VALU load (only RNEA drifts).

usage: python tools/drift.py [launches_per_phase] [--dtype f32|f64] [--packs -1 3 ...]
  --packs: RNEA under each rb_set_tuning("pack", v) in alternation instead of RNEA vs probe
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import bench  # noqa: E402
from rigidbody_amd import ffi  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_lib  # noqa: E402

plib = probe_lib.lib()


def series(launch, n, chunk=100):
    out = []
    for c in range(n // chunk):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(chunk):
            launch(c * chunk + k)
        e1.record()
        e1.synchronize()
        out.append(round(e0.elapsed_time(e1) / chunk * 1e3, 2))
    return out


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=4000)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--packs", nargs="*", type=int, default=None)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    n = a.n
    B = 1 << 20
    dt = bench.DT[a.dtype]
    mb = ffi.Multibody.new()
    mb.upload()
    per = bench.set_bytes(7, B, 4 if a.dtype == "f32" else 8, "rnea")
    nsets = max(2, int(np.ceil(1.25 * (1 << 30) / per)))
    sets = bench.make_sets(mb, B, dt, "rnea", nsets, 20250224, layout="tiled")
    rl = bench.batch_launcher(mb, sets, "rnea", dt, "tiled", B)
    if a.packs:
        res = {}
        for rep in range(a.reps):
            for pk in a.packs:
                ffi.set_tuning("pack", pk)
                rl(0, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                torch.cuda.synchronize()
                s = series(lambda k: rl(k, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), n)
                name = f"pack={pk}#{rep}"
                res[name] = {"us_mean": float(np.mean(s)), "us_min": min(s), "us_max": max(s),
                             "us_p10": float(np.percentile(s, 10)), "us_p90": float(np.percentile(s, 90))}
                print(name, json.dumps(res[name]), flush=True)
        ffi.set_tuning("pack", -1)
        return
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib = ffi.lib()
    pin = [(torch.rand((21, B), device="cuda"), torch.empty((7, B), device="cuda")) for _ in range(nsets)]
    pargs = [(i.data_ptr(), o.data_ptr(), 21, 7, B, B, 1 + 16 * 7, sp) for i, o in pin]

    def probe(k):
        if plib.rb_probe_rows_f32(*pargs[k % nsets]):
            raise RuntimeError(ffi.last_error())

    def rnea(k):
        rl(k, sp)

    res = {}
    for name, f in (("rnea", rnea), ("probe", probe), ("rnea2", rnea), ("probe2", probe)):
        s = series(f, n)
        res[name] = {"us_mean": float(np.mean(s)), "us_min": min(s), "us_max": max(s), "series": s}
        print(name, res[name]["us_mean"], res[name]["us_min"], res[name]["us_max"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
