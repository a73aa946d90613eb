#!/bin/bash
# Round 6: kernarg preload A/B repeated with more rounds (second box)
set -o pipefail
mkdir -p gpurun_out/r6z
V="kernarg_preload=0 kernarg_preload=14 kernarg_preload=0,jit_variant=0"
timeout -k 10 200 python tools/ab_bench.py --kernel rnea --dtype f32 --batch 65536 --graph --layouts tiled --rounds 11 --steps 300 --variants $V > gpurun_out/r6z/ab_rnea32_b65536.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f32 --batch 65536 --graph --layouts tiled --rounds 11 --steps 300 --variants $V > gpurun_out/r6z/ab_fd32_b65536.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch 131072 --graph --layouts tiled --rounds 11 --steps 300 --variants $V > gpurun_out/r6z/ab_idfd64_b131072.log 2>&1 || exit 1
