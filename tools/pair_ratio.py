"""In-process A/B helper: interleaved rounds of several bench workloads (kernel, dtype) on the
tiled layout at one batch size; prints per-workload median kernel us and the ratio to the
first (a clock-independent comparison across boxes).

usage: python tools/pair_ratio.py [--batch 1048576] rnea:f32 fd:f32 fd:f64 ..."""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
import bench  # noqa: E402
from rigidbody_amd import chains, ffi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--steps", type=int, default=1000)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("work", nargs="+")
a = ap.parse_args()
mb = ffi.Multibody.new()
mb.upload()
launch = {}
for w in a.work:
    k, dt = w.split(":")
    es = 4 if dt == "f32" else 8
    ns = bench.nsets_for(mb.n, a.batch, es, k, 1.25)
    sets = bench.make_sets(mb, a.batch, bench.DT[dt], k, ns, chains.SEED, "tiled")
    launch[w] = bench.batch_launcher(mb, sets, k, bench.DT[dt], "tiled", a.batch)
res = {w: [] for w in a.work}
for r in range(a.rounds):
    for w in a.work:
        res[w].append(bench.time_launches(launch[w], a.steps, 20, 1, 200.0 if r == 0 else 20.0)[1] * 1e3)
med = {w: float(np.median(v)) for w, v in res.items()}
base = med[a.work[0]]
print(json.dumps({"batch": a.batch, "us": {w: round(m, 3) for w, m in med.items()},
                  "ratio": {w: round(m / base, 4) for w, m in med.items()}}))
