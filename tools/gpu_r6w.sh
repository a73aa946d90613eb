#!/bin/bash
# Round 6: the role-alternating one-per-lane split (pack 5) against the packed pair above 2^17
set -o pipefail
mkdir -p gpurun_out/r6w
for B in 262144 1048576; do
  timeout -k 10 240 python tools/ab_bench.py --kernel fd --dtype f32 --batch $B --graph --layouts tiled --rounds 7 --steps 100 --variants pack=-1 pack=5 pack=4 > gpurun_out/r6w/ab_fd32_b$B.log 2>&1 || exit 1
  timeout -k 10 240 python tools/ab_bench.py --kernel rnea_fd --dtype f32 --batch $B --graph --layouts tiled --rounds 7 --steps 100 --variants pack=-1 pack=5 > gpurun_out/r6w/ab_idfd32_b$B.log 2>&1 || exit 1
done
