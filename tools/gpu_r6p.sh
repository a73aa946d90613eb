# round 6: non-temporal load / store bits of the fused pair (fd_nt: 1 loads, 2 stores)
set -o pipefail
mkdir -p gpurun_out/r6p
V="fd_nt=3 fd_nt=2 fd_nt=1 fd_nt=0"
timeout -k 10 240 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch 131072 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6p/ab_idfd64s_nt.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --layouts tiled --rounds 7 --steps 200 --variants $V > gpurun_out/r6p/ab_idfd64_nt.log 2>&1 || exit 1
