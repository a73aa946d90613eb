# round 6: rehearsal of the N > 1 bench path with N ranks sharing the one GPU (gloo: RCCL takes one
# rank per device); checks the spawn, the collectives, the config-4 line and the compact JSON at N = 4, 8
set -o pipefail
D=gpurun_out/r6r
mkdir -p $D
for N in 4 8; do
  RB_DIST_BACKEND=gloo RB_BENCH_DETAIL=$D/detail_n$N.json timeout -k 10 400 python bench.py --gpus $N --steps 20 --warmup 5 --rotate-gib 0.6 > $D/bench_n$N.json 2> $D/bench_n$N.err || exit 1
done
