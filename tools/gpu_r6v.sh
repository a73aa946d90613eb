#!/bin/bash
# Round 6: the role-alternating fp32 splits adopted as default -- the full GPU suite, then an
# A/B of the fused pair's split at 2^17 (fp32) and the FD defaults at 2^15..2^17.
set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r6v/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f32 --batch 131072 --graph --layouts tiled --rounds 7 --steps 300 --variants pack=-1 pack=5 > gpurun_out/r6v/ab_idfd32_b131072.log 2>&1 || exit 1
for B in 32768 65536 131072; do
  timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f32 --batch $B --graph --layouts tiled --rounds 7 --steps 300 --variants pack=-1 pack=4 > gpurun_out/r6v/ab_fd32_b$B.log 2>&1 || exit 1
done
