#!/bin/bash
# Round-4 re-profile of the kernels whose defaults changed late in the round: the parked 30-DOF
# fp32 RNEA (bench workload rnea_chain30_f32_tiled_b1048576) and the batched CRBA / Jacobian /
# fwd_kin (tools/q_bench.py, fp64, 2^20).  Same recipe and on-box summaries as
# tools/profile_r04.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TRAFFIC_OUT=gpurun_out/traffic
summ() {  # TAG WORKLOAD [KERNEL_REGEX]
  python3 tools/traffic_summary.py "gpurun_out/$1" "gpurun_out/sum/$1" "$2" ${3:+"$3"} > "gpurun_out/sum_$1.log" 2>&1 || return 1
  find "gpurun_out/$1" -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*agent_info.csv' -delete
}
tools/profile_round.sh c30 --kernel rnea --dtype f32 --dof 30 && summ c30 rnea_chain30_f32_tiled_b1048576 &&
tools/profile_any.sh crba64 tools/q_bench.py --kernel crba --dtype f64 && summ crba64 crba_fr3_f64_soa_b1048576 &&
tools/profile_any.sh jac64 tools/q_bench.py --kernel jac --dtype f64 && summ jac64 jac_fr3_f64_soa_b1048576 &&
tools/profile_any.sh fk64 tools/q_bench.py --kernel fwd_kin --dtype f64 && summ fk64 fwd_kin_fr3_f64_soa_b1048576 &&
python3 tools/clock_probe.py run --seconds 2 --only rnea_chain30_f32 > gpurun_out/clock_probe_c30.jsonl &&
du -sh gpurun_out
