# round 6: LLVM scheduling options of the hipRTC compile (jit_sched), interleaved A/B
set -o pipefail
mkdir -p gpurun_out/r6o
V="jit_sched=0 jit_sched=1 jit_sched=2"
timeout -k 10 240 python tools/ab_bench.py --kernel rnea --dtype f64 --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6o/ab_rnea64.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel fd --dtype f64 --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6o/ab_fd64.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel fd --dtype f32 --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6o/ab_fd32.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch 131072 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6o/ab_idfd64s.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel rnea --dtype f32 --dof 30 --layouts tiled --rounds 5 --steps 200 --variants $V > gpurun_out/r6o/ab_c30.log 2>&1 || exit 1
timeout -k 10 240 python tools/ab_bench.py --kernel fd --dtype f32 --batch 65536 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6o/ab_fd32s.log 2>&1 || exit 1
