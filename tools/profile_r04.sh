#!/bin/bash
# Round-4 profile set (one gpurun call): in-kernel clock / occupancy probes at 2^20 and 65536,
# then tools/profile_round.sh (trace + 5 PMC passes, 300 timed launches each) for every bench
# workload whose counters bench.py reads (profiles/traffic_*.json) and tools/profile_any.sh for
# the fused rollouts.  Each profile is summarised on the box (tools/traffic_summary.py into
# gpurun_out/traffic/ and gpurun_out/sum/TAG/) and its raw per-dispatch CSVs are deleted, so
# what comes back stays far below gpurun's 64 MiB; the kernel-trace stats are kept.
# Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TRAFFIC_OUT=gpurun_out/traffic
summ() {  # TAG WORKLOAD
  python3 tools/traffic_summary.py "gpurun_out/$1" "gpurun_out/sum/$1" "$2" > "gpurun_out/sum_$1.log" 2>&1 || return 1
  find "gpurun_out/$1" -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*agent_info.csv' -delete
}
prof() {  # TAG WORKLOAD bench args...
  local tag=$1 wl=$2; shift 2
  tools/profile_round.sh "$tag" "$@" && summ "$tag" "$wl"
}
profany() {  # TAG WORKLOAD script args...
  local tag=$1 wl=$2; shift 2
  tools/profile_any.sh "$tag" "$@" && summ "$tag" "$wl"
}
tools/gpu_steps.sh \
  clock_probe 200 "python3 tools/clock_probe.py run --seconds 2 > gpurun_out/clock_probe.jsonl" \
  clock_probe_b65536 200 "python3 tools/clock_probe.py run --seconds 2 --batch 65536 > gpurun_out/clock_probe_b65536.jsonl" &&
prof rnea64 rnea_fr3_f64_tiled_b1048576 &&
prof fd64 fd_fr3_f64_tiled_b1048576 --kernel fd --dtype f64 &&
prof fd32 fd_fr3_f32_tiled_b1048576 --kernel fd --dtype f32 &&
prof c30 rnea_chain30_f32_tiled_b1048576 --kernel rnea --dtype f32 --dof 30 &&
prof rnea32 rnea_fr3_f32_tiled_b1048576 --kernel rnea --dtype f32 &&
prof fd32s fd_fr3_f32_tiled_b65536 --kernel fd --dtype f32 --batch 65536 &&
prof rnea32s rnea_fr3_f32_tiled_b65536 --kernel rnea --dtype f32 --batch 65536 &&
profany roll32 rollout_fr3_f32_K16_b1048576 tools/ab_bench.py --kernel rollout --dtype f32 --variants pack=-1 --rounds 2 --steps 20 &&
profany roll64 rollout_fr3_f64_K16_b1048576 tools/ab_bench.py --kernel rollout --dtype f64 --variants pack=-1 --rounds 2 --steps 20 &&
du -sh gpurun_out
