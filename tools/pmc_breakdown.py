"""Per-wave cycle breakdown and HBM traffic of one profiled kernel, from the committed PMC
summaries under profiles/<round>/<kernel>/ (pmc_sq_summary.csv, pmc_fetch_summary.csv,
pmc_write_summary.csv, kernel_stats.csv as tools/profile_round.sh writes them).

SQ_* cycle counters on gfx950 count quad-cycles (x4 = shader-clock cycles); FETCH_SIZE and
WRITE_SIZE are KB per launch, traffic = 2 * FETCH + WRITE (MI355X_MICROARCH.md's gfx950
correction).  usage: python tools/pmc_breakdown.py profiles/r02/fd32 [algorithmic_bytes [clock_GHz]]
clock_GHz: the in-kernel clock the chip holds under this kernel (tools/clock_probe.py); the
VALU floor is then also priced at that clock instead of the 2.4 GHz maximum.
"""
import csv
import os
import sys


def read(path):
    with open(path) as f:
        return {r["counter"]: float(r["mean_per_launch"]) for r in csv.DictReader(f)}


def kernel_avg_us(path):
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if r["Name"] == "rb_jit_kernel"]
    return float(rows[0]["AverageNs"]) / 1e3 if rows else None


def breakdown(d, algo_bytes=None, clock_ghz=None):
    sq = read(os.path.join(d, "pmc_sq_summary.csv"))
    w = sq["SQ_WAVES"]
    out = {
        "waves": int(w),
        "cycles_per_wave": 4 * sq["SQ_WAVE_CYCLES"] / w,
        "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / w,
        "valu_issue_cycles_per_wave": 4 * sq["SQ_ACTIVE_INST_VALU"] / w,
        "dependency_wait_cycles_per_wave": 4 * sq["SQ_WAIT_INST_ANY"] / w,
        "any_wait_cycles_per_wave": 4 * sq["SQ_WAIT_ANY"] / w,
    }
    f, wr = os.path.join(d, "pmc_fetch_summary.csv"), os.path.join(d, "pmc_write_summary.csv")
    if os.path.exists(f) and os.path.exists(wr):
        t = (2 * read(f)["FETCH_SIZE"] + read(wr)["WRITE_SIZE"]) * 1024
        out["hbm_traffic_MB"] = t / 1e6
        if algo_bytes:
            out["traffic_over_algorithmic"] = t / algo_bytes
    ks = os.path.join(d, "kernel_stats.csv")
    if os.path.exists(ks):
        out["trace_kernel_us_avg"] = kernel_avg_us(ks)
    # VALU-issue floor: every SIMD issues its waves' VALU back to back (1024 SIMDs, 2.4 GHz)
    out["valu_floor_us"] = out["valu_issue_cycles_per_wave"] * w / 1024 / 2.4e3
    if clock_ghz:
        out["valu_floor_us_at_held_clock"] = out["valu_issue_cycles_per_wave"] * w / 1024 / (clock_ghz * 1e3)
    if algo_bytes:
        out["algorithmic_MB"] = algo_bytes / 1e6
        # memory floor at the no-math probe's ceiling for this access pattern (5.97 TB/s)
        out["pattern_floor_us"] = algo_bytes / 5.97e12 * 1e6
    return out


def main():
    d = sys.argv[1]
    algo = float(sys.argv[2]) if len(sys.argv) > 2 else None
    clock = float(sys.argv[3]) if len(sys.argv) > 3 else None
    for k, v in breakdown(d, algo, clock).items():
        print(f"{k:34s} {v:.4g}" if isinstance(v, float) else f"{k:34s} {v}")


if __name__ == "__main__":
    main()
