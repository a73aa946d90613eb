#!/bin/bash
# Round 6: raised wave priority while a lane issues its rows (RB_VARIANT bit 262144), headline
# (the A/B selector was removed after this run, DESIGN.md §10: rejected)
set -o pipefail
mkdir -p gpurun_out/r6q
timeout -k 10 400 python tools/ab_bench.py --kernel rnea --dtype f64 --batch 1048576 --layouts tiled --rounds 9 --steps 100 --variants jit_variant=0 jit_variant=262144 jit_variant=262144,jit_waves=4 > gpurun_out/r6q/ab_rnea64_prio.log 2>&1 || exit 1
