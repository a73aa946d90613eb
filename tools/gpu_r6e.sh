# round 6: headline fp64 RNEA launch-shape sweep (interleaved A/B, one process)
set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 300 python tools/ab_bench.py --kernel rnea --dtype f64 --layouts tiled --rounds 7 --steps 400 \
  --variants pack=-1 pack=1 seq_tail=0 seq_tail=50 seq_tail=100 rnea_nt=0 > gpurun_out/r6e/ab_rnea64_shapes.log 2>&1
