#!/bin/bash
# Round 6: wave priority by role in the fp32 FD one-per-lane split (RB_VARIANT 524288: mass-matrix
# wave raised, 1048576: bias wave raised), config 3 size and 2^17
# (the A/B selectors were removed after this run, DESIGN.md §10: rejected)
set -o pipefail
mkdir -p gpurun_out/r6s
for B in 65536 131072; do
  timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f32 --batch $B --graph --layouts tiled --rounds 9 --steps 300 --variants jit_variant=0 jit_variant=524288 jit_variant=1048576 > gpurun_out/r6s/ab_fd32_prio_b$B.log 2>&1 || exit 1
done
