# round 6: fp32 fused pair forms (one per lane / packed pair / wave split) by batch size
set -o pipefail
mkdir -p gpurun_out/r6l
for B in 65536 131072 262144 1048576; do
  timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f32 --batch $B --graph --layouts tiled --rounds 5 --steps 300 --variants pack=1 pack=2 pack=5 > gpurun_out/r6l/ab_idfd32_b$B.log 2>&1 || exit 1
done
