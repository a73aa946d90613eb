# round 6: fp32 FD wave split at small batches: roles alternated per block (jit_variant 131072)
set -o pipefail
mkdir -p gpurun_out/r6u
for B in 32768 65536 131072; do
  timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f32 --batch $B --graph --layouts tiled --rounds 7 --steps 300 --variants pack=-1 pack=5 pack=5,jit_variant=131072 pack=4 > gpurun_out/r6u/ab_fd32_mix_b$B.log 2>&1 || exit 1
done
for B in 32768 65536; do
  timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f32 --batch $B --graph --layouts tiled --rounds 7 --steps 300 --variants pack=-1 pack=5,jit_variant=131072 > gpurun_out/r6u/ab_idfd32_mix_b$B.log 2>&1 || exit 1
done
