"""Attribute the one-per-lane fp64 RNEA's slow/fast phases from per-dispatch PMC:
splits the profiled headline dispatches into fast / slow by their own duration and reports, per
group, the mean duration and counters per dispatch -- GRBM_GUI_ACTIVE / ns (an effective-clock
proxy: the counter is summed over the chip's GRBM instances) and the SQ wave-time split.

usage: python tools/phase_pmc.py PMC_DIR [KERNEL]   (a rocprofv3 --pmc ... -d PMC_DIR run)"""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "rb_jit_kernel"
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] != kern:
                continue
            key = int(r["Dispatch_Id"])
            e = rows.setdefault(key, {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ds = [rows[k] for k in sorted(rows)][-4000:]
    dur = np.array([x["dur_ns"] for x in ds], float)
    thr = float(np.percentile(dur, 50))
    out = {"dispatches": len(ds), "duration_ns_p10_p50_p90": [float(np.percentile(dur, p)) for p in (10, 50, 90)]}
    lo, hi = np.percentile(dur, 25), np.percentile(dur, 75)
    for name, sel in (("fast_quartile", dur <= lo), ("slow_quartile", dur >= hi)):
        g = [x for x, s in zip(ds, sel) if s]
        keys = sorted(k for k in g[0] if k != "dur_ns")
        agg = {"n": len(g), "dur_ns": float(np.mean([x["dur_ns"] for x in g]))}
        for k in keys:
            agg[k] = float(np.mean([x[k] for x in g]))
        if "GRBM_GUI_ACTIVE" in agg:
            agg["GRBM_GUI_ACTIVE_per_ns"] = agg["GRBM_GUI_ACTIVE"] / agg["dur_ns"]
        out[name] = agg
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
