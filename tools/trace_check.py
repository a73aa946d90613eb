"""Agreement check between bench.py's hipEvent timing and rocprofv3's kernel trace of the SAME
process (tools/profile_round.sh `trace` step): the headline JSON line that process printed vs
the mean duration of the last `steps` headline-kernel dispatches in its kernel trace (the
timed region), plus the idle gap between them.

usage: python tools/trace_check.py BENCH_LOG TRACE_DIR OUT_JSON
  (tools/profile_round.sh TAG: gpurun_out/TAG_trace.log and gpurun_out/TAG/trace)
"""
import csv
import glob
import json
import os
import sys


def main():
    log, tdir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    line = None
    for ln in open(log):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    steps = line["steps"]
    f = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                  for r in csv.DictReader(open(f)) if r["Kernel_Name"] == "rb_jit_kernel")
    timed = rows[-steps:]
    dur = [(e - s) / 1e3 for s, e in timed]
    gaps = [(timed[i + 1][0] - timed[i][1]) / 1e3 for i in range(len(timed) - 1)]
    alld = [(e - s) / 1e3 for s, e in rows]
    chunk = max(1, steps // 8)
    rf = line["roofline"]
    bytes_launch = rf["bytes_per_eval"] * rf["evals_per_launch"]
    peak = rf["peak"] * 1e9
    win = sum(dur) / len(dur)
    # the timed window as the hipEvent pair sees it: first start to last end over `steps` launches
    span = (timed[-1][1] - timed[0][0]) / 1e3 / steps
    res = {
        "workload": line["config"]["workload"],
        "steps": steps,
        "bench_kernel_us_avg (hipEvent pair / steps)": rf["kernel_ms_avg"] * 1e3,
        "bench_ms_per_step_us (wall / steps)": line["ms_per_step"] * 1e3,
        "bench_roofline_frac": rf["frac"],
        "trace_kernel_us_avg (last `steps` dispatches)": win,
        "trace_window_span_us (first start .. last end / steps)": span,
        "trace_gap_us_avg": sum(gaps) / max(1, len(gaps)),
        "trace_period_us": (timed[-1][0] - timed[0][0]) / 1e3 / max(1, steps - 1),
        "trace_kernel_us_by_eighth": [round(sum(dur[k:k + chunk]) / len(dur[k:k + chunk]), 2)
                                      for k in range(0, len(dur), chunk)],
        "all_dispatches": len(rows),
        "trace_kernel_us_avg_all_dispatches (spin-up and warmup included)": sum(alld) / len(alld),
        "algorithmic_bytes_per_launch": bytes_launch,
        "frac_from_trace_window_mean": bytes_launch / (win * 1e-6) / peak,
        "frac_from_trace_window_span": bytes_launch / (span * 1e-6) / peak,
    }
    res["check"] = {
        "window_span_within_3pct_of_bench_frac":
            abs(res["frac_from_trace_window_span"] / rf["frac"] - 1) <= 0.03,
        "window_mean_le_ms_per_step": win <= line["ms_per_step"] * 1e3,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
