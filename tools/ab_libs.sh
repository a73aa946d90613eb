#!/bin/bash
# Same-box A/B of two builds of the library (e.g. ab/lib_r03.so vs the in-tree one): runs the
# given bench.py arguments alternately under each, ROUNDS times, one JSON line per run in
# gpurun_out/ab_libs_<tag>.jsonl.  usage: tools/ab_libs.sh TAG ROUNDS OLD.so -- bench args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; rounds=$2; old=$3; shift 4
mkdir -p gpurun_out
out=gpurun_out/ab_libs_$tag.jsonl
: > "$out"
for r in $(seq 1 "$rounds"); do
  for which in old new; do
    if [ $which = old ]; then lib=$old; else lib=rigidbody-rs_amd/librigidbody_bindings.so; fi
    line=$(RIGIDBODY_AMD_LIB=$PWD/$lib timeout -k 10 240 python bench.py "$@" 2>gpurun_out/ab_libs_${tag}_err.log | tail -n 1)
    rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc on $which round $r"; cat gpurun_out/ab_libs_${tag}_err.log | tail -5; exit $rc; }
    echo "{\"lib\": \"$which\", \"round\": $r, \"line\": $line}" >> "$out"
    echo "$which r$r: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1000, "us", d.get("roofline",{}).get("frac"))')"
  done
done
