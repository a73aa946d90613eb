"""Per-kernel duration groups from a rocprofv3 SQLite (rocpd) result: consecutive dispatches of the
same kernel / grid / VGPR count / LDS size, with their median and minimum durations.

usage: python tools/trace_groups.py RESULTS.db [min_count]"""
import itertools
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    mincount = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rows = list(c.execute("select name, start, end, grid_x, vgpr_count, lds_size from kernels order by start"))
    for key, grp in itertools.groupby(rows, key=lambda r: (r[0][:40], r[3], r[4], r[5])):
        d = sorted((r[2] - r[1]) / 1e3 for r in grp)
        if len(d) >= mincount:
            print(f"{key[0]:40s} grid {key[1]:8d} vgpr {key[2]:3d} lds {key[3]:6d}  n {len(d):6d}  "
                  f"median {d[len(d) // 2]:8.3f} us  min {d[0]:8.3f}")


if __name__ == "__main__":
    main()
