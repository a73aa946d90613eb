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
    f = glob.glob(os.path.join(tdir, "*kernel_trace.csv"))[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                  for r in csv.DictReader(open(f)) if r["Kernel_Name"] == "rb_jit_kernel")
    timed = rows[-steps:]
    dur = [(e - s) / 1e3 for s, e in timed]
    gaps = [(timed[i + 1][0] - timed[i][1]) / 1e3 for i in range(len(timed) - 1)]
    chunk = max(1, steps // 8)
    res = {
        "workload": line["config"]["workload"],
        "steps": steps,
        "bench_kernel_us_avg (hipEvent pair / steps)": line["roofline"]["kernel_ms_avg"] * 1e3,
        "trace_kernel_us_avg (last `steps` dispatches)": sum(dur) / len(dur),
        "trace_gap_us_avg": sum(gaps) / max(1, len(gaps)),
        "trace_period_us": (timed[-1][0] - timed[0][0]) / 1e3 / max(1, steps - 1),
        "trace_kernel_us_by_eighth": [round(sum(dur[k:k + chunk]) / len(dur[k:k + chunk]), 2)
                                      for k in range(0, len(dur), chunk)],
        "all_dispatches": len(rows),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
