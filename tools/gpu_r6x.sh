#!/bin/bash
# Round 6: the 30-link fp32 RNEA (config 5) -- the reversed sweep (rnea_rev = 2, 5 waves/SIMD,
# +27% VALU) against the parked form (3 waves/SIMD)
# (the A/B selector was removed after this run, DESIGN.md §10: rejected)
set -o pipefail
mkdir -p gpurun_out/r6x
timeout -k 10 300 python tools/ab_bench.py --kernel rnea --dtype f32 --dof 30 --batch 1048576 --layouts tiled soa --rounds 5 --steps 50 --variants rnea_rev=-1 rnea_rev=2 > gpurun_out/r6x/ab_c30_f32_rev.log 2>&1 || exit 1
