"""Summarise rocprofv3 PMC passes of the headline kernel into profiles/.

usage: python tools/traffic_summary.py GPURUN_OUT_DIR PROFILE_DIR WORKLOAD [KERNEL_REGEX]

Reads <dir>/pmc_fetch/*counter_collection.csv, pmc_write/…, pmc_sq/…, pmc_grbm/…, pmc_flops/… (one
rocprofv3 --pmc pass each: FETCH_SIZE costs 3 TCC slots and WRITE_SIZE 2, so they cannot
share a pass, MI355X_MICROARCH.md "rocprofv3 PMC slots") and writes
  PROFILE_DIR/pmc_<pass>_summary.csv    per-counter mean / min / max / launches
  profiles/traffic_<WORKLOAD>.json      the HBM bytes bench.py reports as roofline.traffic
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024): gfx950 FETCH_SIZE counts half
the bytes of a coalesced streaming read -- calibrated on this repo's generic RNEA kernel
(exactly 88.08 MB read -> 43 064 KB) and on the device fill (29.36 MB written -> 28 672 KB).
"""
import csv
import glob
import json
import os
import sys


def load(d, regex, durations=None):
    import re
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if re.search(regex, r["Kernel_Name"]):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                if durations is not None and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    durations.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals


def main():
    src, prof, workload = sys.argv[1:4]
    regex = sys.argv[4] if len(sys.argv) > 4 else "rb_jit_kernel"
    os.makedirs(prof, exist_ok=True)
    per = {}
    durs = []
    grbm = []
    for p in ("fetch", "write", "sq", "grbm", "flops"):
        v = load(os.path.join(src, f"pmc_{p}"), regex, durs if p == "grbm" else None)
        if p == "grbm":
            grbm = v.get("GRBM_GUI_ACTIVE", [])
        if not v:
            continue
        with open(os.path.join(prof, f"pmc_{p}_summary.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["counter", "mean_per_launch", "min", "max", "launches"])
            for k, xs in sorted(v.items()):
                w.writerow([k, sum(xs) / len(xs), min(xs), max(xs), len(xs)])
                per[k] = sum(xs) / len(xs)
    model = workload.split("_")[1] if workload.startswith(("rnea_", "fd_")) else "fr3"
    n = 7 if model == "fr3" else int(model[5:]) if model.startswith("chain") else 7
    B = int(workload.rsplit("_b", 1)[1])
    es = 4 if "_f32_" in workload else 8
    alg = (6 if workload.startswith("rnea_fd") else 4) * n * es * B  # rnea_fd: q, qd, qdd, tau_in -> tau, qdd'
    q_rows = {"crba": n * n, "jac": 6 * n, "fwd": 3}.get(workload.split("_")[0])
    if q_rows is not None:  # q-only kernels: n rows read, n*n / 6n / 3 rows written
        alg = (n + q_rows) * es * B
    if workload.startswith("rollout_"):  # K steps: K tau rows read, q and qd read and written
        K = int(workload.split("_K")[1].split("_")[0])
        alg = (K + 4) * n * es * B
    kind = workload.split("_")[0]
    out = {"workload": workload, "kernel": f"{regex} (model-specialised {kind.upper()})",
           "algorithmic_bytes_per_launch": alg}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        hbm = 2 * per["FETCH_SIZE"] * 1024 + per["WRITE_SIZE"] * 1024
        out.update({"bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / alg,
                    "FETCH_SIZE_KB_per_launch": per["FETCH_SIZE"], "WRITE_SIZE_KB_per_launch": per["WRITE_SIZE"]})
    sq = {k: v for k, v in per.items() if k.startswith("SQ_")}
    out["sq_counters_per_launch"] = sq
    if "SQ_WAVE_CYCLES" in sq and sq["SQ_WAVE_CYCLES"] > 0:
        # quad-cycle counters (MI355X_MICROARCH.md): fractions of the waves' lifetime
        wc = sq["SQ_WAVE_CYCLES"]
        out["wave_time_fractions"] = {k.replace("SQ_", "").lower(): sq[k] / wc for k in
                                      ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")
                                      if k in sq}
        if "SQ_WAVES" in sq:
            out["valu_insts_per_wave"] = sq.get("SQ_INSTS_VALU", 0) / sq["SQ_WAVES"]
    if grbm and durs:
        # GRBM_GUI_ACTIVE per ns of the (serialised, profiled) dispatch: a relative clock /
        # busy measure per launch window; the per-eighth profile attributes slow phases
        k = max(1, len(grbm) // 8)
        rate = [g / d for g, d in zip(grbm, durs)]
        out["grbm_gui_active_per_ns"] = {
            "mean": sum(rate) / len(rate),
            "by_eighth": [round(sum(rate[i:i + k]) / len(rate[i:i + k]), 3) for i in range(0, len(rate), k)],
            "dispatch_ns_by_eighth": [round(sum(durs[i:i + k]) / len(durs[i:i + k]), 1) for i in range(0, len(durs), k)],
            "note": "GRBM_GUI_ACTIVE / (End - Start) of the PMC pass's dispatches (counter summed over the "
                    "chip's GRBM instances, so a relative figure, not MHz)"}
    out["grbm_per_launch"] = {k: v for k, v in per.items() if k.startswith("GRBM_")}
    fl = {k: v for k, v in per.items() if k.startswith("SQ_INSTS_VALU_FLOPS")}
    if fl:
        # gfx950 FLOP counters (pass pmc_flops): FLOPs the kernel's VALU executed per launch
        out["valu_flops_per_launch"] = fl
    out["method"] = ("rocprofv3 --pmc passes FETCH_SIZE / WRITE_SIZE / SQ_* / GRBM_* / SQ_INSTS_VALU_FLOPS_* run separately on "
                     "`bench.py --no-cpu-baseline --no-secondary`, kernels matching " + regex +
                     ", mean over the profiled launches; bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), "
                     "gfx950 FETCH_SIZE halving calibrated as this script's docstring says")
    # TRAFFIC_OUT: where traffic_<workload>.json goes (default profiles/; on the GPU box a
    # directory under gpurun_out/, which is what comes back)
    dest = os.environ.get("TRAFFIC_OUT", "profiles")
    os.makedirs(dest, exist_ok=True)
    with open(os.path.join(dest, f"traffic_{workload}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in out if k not in ("sq_counters_per_launch", "grbm_per_launch", "method")}))


if __name__ == "__main__":
    main()
