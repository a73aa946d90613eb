#!/bin/bash
# Same-box A/B of two builds: a frozen copy of an earlier tree's bench.py + Python package +
# library (e.g. ab/r03/, from `git worktree add`) against the current tree, alternately, ROUNDS
# times, one JSON line per run in gpurun_out/ab_libs_<tag>.jsonl.
# usage: tools/ab_libs.sh TAG ROUNDS OLD_TREE -- bench args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; rounds=$2; old=$3; shift 4
mkdir -p gpurun_out
out=gpurun_out/ab_libs_$tag.jsonl
: > "$out"
for r in $(seq 1 "$rounds"); do
  for which in old new; do
    if [ $which = old ]; then b=$old/bench.py; else b=bench.py; fi
    line=$(timeout -k 10 240 python "$b" "$@" 2>gpurun_out/ab_libs_${tag}_${which}_err.log | tail -n 1)
    rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc on $which round $r"; tail -5 gpurun_out/ab_libs_${tag}_${which}_err.log; exit $rc; }
    [ -z "$line" ] && { echo "no line from $which round $r"; tail -5 gpurun_out/ab_libs_${tag}_${which}_err.log; exit 1; }
    echo "{\"lib\": \"$which\", \"round\": $r, \"line\": $line}" >> "$out"
    echo "$which r$r: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000, 2), "us", round(d["roofline"]["frac"], 3))')"
  done
done
