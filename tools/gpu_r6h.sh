# round 6: fused pair, early loads of qdd / tau_in (jit_variant 65536) vs after the bias sweep
set -o pipefail
mkdir -p gpurun_out/r6h
for B in 131072 262144 1048576; do
  timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch $B --graph --layouts tiled --rounds 5 --steps 400 --variants jit_variant=0 jit_variant=65536 > gpurun_out/r6h/ab_idfd64_early_b$B.log 2>&1 || exit 1
done
