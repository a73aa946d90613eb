"""Per-launch mean of each PMC counter of one kernel from a rocprofv3 --pmc run's SQLite output
(run_results.db), over the last N dispatches.  usage: python tools/pmc_db_summary.py DB [KERNEL_RE] [N]"""
import collections
import json
import re
import sqlite3
import sys

db = sys.argv[1]
kre = re.compile(sys.argv[2] if len(sys.argv) > 2 else "rb_jit_kernel")
last = int(sys.argv[3]) if len(sys.argv) > 3 else 10
con = sqlite3.connect(db)
per = collections.defaultdict(dict)
for disp, name, c, v, dur in con.execute(
        "select dispatch_id, kernel_name, counter_name, sum(value), max(duration) from counters_collection "
        "group by dispatch_id, counter_name"):
    if kre.search(name):
        per[disp][c] = v
        per[disp]["duration_ns"] = dur
ks = sorted(per)[-last:]
mean = {c: sum(per[k][c] for k in ks) / len(ks) for c in per[ks[0]]}
print(json.dumps({"db": db, "kernel_re": kre.pattern, "dispatches": len(per), "averaged": len(ks), "mean": mean}, indent=1))
