#!/bin/bash
# The committed-profile recipe (one gpurun call): for each named workload, a kernel trace and the
# PMC passes of tools/profile_round.sh (bench.py workloads) or tools/profile_any.sh (rollouts,
# q-only queries), summarised on the box into profiles/traffic_*.json form
# (tools/traffic_summary.py -> gpurun_out/traffic/ and gpurun_out/sum/TAG/); the raw per-dispatch
# CSVs are deleted so what comes back stays far below gpurun's 64 MiB (kernel-trace stats kept).
# `clock` runs the in-kernel clock / occupancy probes (tools/clock_probe.py).  Stops at the first
# failing step.
#
# usage (via gpurun): tools/profile_set.sh NAME...
#   NAME in: clock rnea64 rnea32 rnea32s fd64 idfd64 idfd64s fd32 fd32s c30 c30_64 roll32 roll64
#            crba64 jac64 fk64 crba64t jac64t fk64t
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TRAFFIC_OUT=gpurun_out/traffic
summ() {  # TAG WORKLOAD
  python3 tools/traffic_summary.py "gpurun_out/$1" "gpurun_out/sum/$1" "$2" > "gpurun_out/sum_$1.log" 2>&1 || return 1
  find "gpurun_out/$1" -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*agent_info.csv' -delete
}
prof() {  # TAG WORKLOAD bench args...
  local tag=$1 wl=$2; shift 2
  # trace_check before summ deletes the per-dispatch trace: the traced run's own bench line against
  # the mean of its last `steps` dispatches (the timed window) and the all-dispatch mean
  tools/profile_round.sh "$tag" "$@" &&
    mkdir -p "gpurun_out/sum/$tag" &&
    python3 tools/trace_check.py "gpurun_out/${tag}_trace.log" "gpurun_out/$tag/trace" \
      "gpurun_out/sum/$tag/trace_window.json" > /dev/null &&
    summ "$tag" "$wl"
}
profany() {  # TAG WORKLOAD script args...
  local tag=$1 wl=$2; shift 2
  tools/profile_any.sh "$tag" "$@" && summ "$tag" "$wl"
}
one() {
  case $1 in
    clock) tools/gpu_steps.sh \
             clock_probe 200 "python3 tools/clock_probe.py run --seconds 2 > gpurun_out/clock_probe.jsonl" \
             clock_probe_b65536 200 "python3 tools/clock_probe.py run --seconds 2 --batch 65536 > gpurun_out/clock_probe_b65536.jsonl" ;;
    rnea64) prof rnea64 rnea_fr3_f64_tiled_b1048576 ;;
    rnea32) prof rnea32 rnea_fr3_f32_tiled_b1048576 --kernel rnea --dtype f32 ;;
    rnea32s) prof rnea32s rnea_fr3_f32_tiled_b65536 --kernel rnea --dtype f32 --batch 65536 ;;
    fd64) prof fd64 fd_fr3_f64_tiled_b1048576 --kernel fd --dtype f64 ;;
    idfd64) prof idfd64 rnea_fd_fr3_f64_tiled_b1048576 --kernel rnea_fd --dtype f64 ;;
    idfd64s) prof idfd64s rnea_fd_fr3_f64_tiled_b131072 --kernel rnea_fd --dtype f64 --batch 131072 ;;
    fd32) prof fd32 fd_fr3_f32_tiled_b1048576 --kernel fd --dtype f32 ;;
    fd32s) prof fd32s fd_fr3_f32_tiled_b65536 --kernel fd --dtype f32 --batch 65536 ;;
    c30) prof c30 rnea_chain30_f32_tiled_b1048576 --kernel rnea --dtype f32 --dof 30 ;;
    c30_64) prof c30_64 rnea_chain30_f64_tiled_b1048576 --kernel rnea --dtype f64 --dof 30 ;;
    roll32) profany roll32 rollout_fr3_f32_K16_b1048576 tools/ab_bench.py --kernel rollout --dtype f32 \
              --variants pack=-1 --rounds 2 --steps 20 ;;
    roll64) profany roll64 rollout_fr3_f64_K16_b1048576 tools/ab_bench.py --kernel rollout --dtype f64 \
              --variants pack=-1 --rounds 2 --steps 20 ;;
    crba64|jac64|fk64|crba64t|jac64t|fk64t)
      local k=${1%t} lay=soa
      [ "${1: -1}" = t ] && lay=tiled
      k=${k%64}
      local kern=$k
      [ "$k" = fk ] && kern=fwd_kin
      profany "$1" "${kern}_fr3_f64_${lay}_b1048576" tools/q_bench.py --kernel "$kern" --dtype f64 --layout "$lay" ;;
    *) echo "unknown workload $1"; return 2 ;;
  esac
}
for name in "$@"; do
  one "$name" || exit $?
done
du -sh gpurun_out
