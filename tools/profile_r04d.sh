#!/bin/bash
# Round-4 profile of the tiled-layout q-only entry points (multibody_{crba,jac,fwd_kin}_batch_tiled_f64,
# tools/q_bench.py --layout tiled, FR3 2^20): kernel trace + the PMC passes of tools/profile_any.sh,
# summarised on the box into profiles/traffic_*.json form (tools/traffic_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TRAFFIC_OUT=gpurun_out/traffic
summ() {  # TAG WORKLOAD
  python3 tools/traffic_summary.py "gpurun_out/$1" "gpurun_out/sum/$1" "$2" > "gpurun_out/sum_$1.log" 2>&1 || return 1
  find "gpurun_out/$1" -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*agent_info.csv' -delete
}
tools/profile_any.sh crba64t tools/q_bench.py --kernel crba --dtype f64 --layout tiled && summ crba64t crba_fr3_f64_tiled_b1048576 &&
tools/profile_any.sh jac64t tools/q_bench.py --kernel jac --dtype f64 --layout tiled && summ jac64t jac_fr3_f64_tiled_b1048576 &&
tools/profile_any.sh fk64t tools/q_bench.py --kernel fwd_kin --dtype f64 --layout tiled && summ fk64t fwd_kin_fr3_f64_tiled_b1048576 &&
du -sh gpurun_out
