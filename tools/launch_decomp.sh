#!/bin/bash
# GPU-box recipe: kernel traces of HIP-graph replays of the config-2 / config-3 launches (FR3,
# 65536 configurations, fp32, tiled) and their per-launch period / busy / gap decomposition
# (tools/launch_decomp.py).  Outputs gpurun_out/launch_decomp/{rnea,fd}/ + summary.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
O=$R/gpurun_out/launch_decomp
mkdir -p "$O"
export TMPDIR=/tmp
: > "$O/summary.jsonl"
for k in rnea fd; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/$k" -o run -- \
     python3 "$R/tools/launch_decomp.py" run --kernel $k --dtype f32 --batch 65536) > "$O/$k.log" 2>&1 || exit $?
  line=$(grep '^{' "$O/$k.log" | tail -n 1)
  dec=$(python3 "$R/tools/launch_decomp.py" analyze "$O/$k")
  echo "{\"kernel\": \"$k\", \"run\": $line, \"trace\": $dec}" | tee -a "$O/summary.jsonl"
done
