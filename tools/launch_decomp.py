"""Per-launch cost of the small-batch configs (FR3, B = 65536), from
a rocprofv3 kernel trace of HIP-graph replays of the C-ABI launches (the device-bound rate bench.py
reports as *_graph).

  run:      python tools/launch_decomp.py run [--kernel fd] [--dtype f32] [--batch 65536]
            (under `rocprofv3 --kernel-trace --output-format csv -- python ...`): captures 100
            consecutive launches over rotating input sets in one HIP graph, replays it 20 times.
  analyze:  python tools/launch_decomp.py analyze TRACE_DIR [--name rb_jit_kernel]
            For consecutive dispatches of the kernel inside one replay (gap < 50 us):
              period   = start(i+1) - start(i)            (what one launch costs the stream)
              busy     = end(i) - start(i)                (dispatch begin to completion signal:
                                                            first wave start .. last wave end plus
                                                            the dispatch / completion overhead)
              gap      = start(i+1) - end(i)              (between one kernel's completion and the
                                                            next one's start: the per-launch cost
                                                            the device pays between graph nodes)
            medians / p10 / p90 in us, one JSON line.
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np


def run(a):
    import torch

    REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    sys.path[:0] = [REPO, os.path.join(REPO, "rigidbody-rs_amd")]
    import bench
    from rigidbody_amd import chains, ffi

    mb = ffi.Multibody.new()
    mb.upload()
    dtype = bench.DT[a.dtype]
    es = 4 if a.dtype == "f32" else 8
    ns = bench.nsets_for(mb.n, a.batch, es, a.kernel, 1.25)
    sets = bench.make_sets(mb, a.batch, dtype, a.kernel, ns, chains.SEED, a.layout)
    launch = bench.batch_launcher(mb, sets, a.kernel, dtype, a.layout, a.batch)
    wall, ms, n = bench.time_graph(launch, 100 * a.replays)
    print(json.dumps({"kernel": a.kernel, "dtype": a.dtype, "batch": a.batch, "layout": a.layout,
                      "graph_us_per_launch": ms * 1e3, "launches": n,
                      "kernel_form": mb.kernel_form(a.kernel, a.dtype == "f64", a.batch, a.layout == "tiled")}))


def analyze(a):
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if a.name in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    period, busy, gap = [], [], []
    for (s0, e0), (s1, _) in zip(rows, rows[1:]):
        if s1 - e0 > 50_000:  # between replays / outside a replay
            continue
        period.append((s1 - s0) / 1e3)
        busy.append((e0 - s0) / 1e3)
        gap.append((s1 - e0) / 1e3)

    def st(x):
        x = np.asarray(x)
        return {"median": round(float(np.median(x)), 3), "p10": round(float(np.percentile(x, 10)), 3),
                "p90": round(float(np.percentile(x, 90)), 3)}

    print(json.dumps({"dispatches": len(rows), "pairs": len(period), "period_us": st(period), "busy_us": st(busy),
                      "gap_us": st(gap)}))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--kernel", default="fd")
    r.add_argument("--dtype", default="f32")
    r.add_argument("--batch", type=int, default=65536)
    r.add_argument("--layout", default="tiled")
    r.add_argument("--replays", type=int, default=20)
    z = sub.add_parser("analyze")
    z.add_argument("dir")
    z.add_argument("--name", default="rb_jit_kernel")
    a = ap.parse_args()
    (run if a.cmd == "run" else analyze)(a)


if __name__ == "__main__":
    main()
