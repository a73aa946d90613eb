#!/bin/bash
# Round-4 re-profile of the fp32 FR3 RNEA at 2^20 on the tiled layout after it dropped its
# non-temporal loads / stores (tuning rnea_nt auto), then a driver-style bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TRAFFIC_OUT=gpurun_out/traffic
tools/profile_round.sh rnea32 --kernel rnea --dtype f32 &&
python3 tools/traffic_summary.py gpurun_out/rnea32 gpurun_out/sum/rnea32 rnea_fr3_f32_tiled_b1048576 > gpurun_out/sum_rnea32.log 2>&1 &&
find gpurun_out/rnea32 -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*agent_info.csv' -delete &&
tools/gpu_steps.sh bench_driver 400 "python3 bench.py --gpus 1 --steps 20 --warmup 5"
