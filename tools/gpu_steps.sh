#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# Continues after an ordinary failure (exit 1-2, e.g. a failed assertion) so one call
# reports everything; stops at once after a fault, abort, kill or timeout
# (124/134/137/139 or >128), as the GPU pool requires.
# usage: tools/gpu_steps.sh name1 secs1 'cmd1' name2 secs2 'cmd2' ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc after $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -ge 124 ]; then echo "!! stopping: fault/timeout in $name"; exit $rc; fi
done
exit $status
