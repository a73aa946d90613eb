#!/bin/bash
# Round 6: kernel-argument preload (-amdgpu-kernarg-preload-count) on the hipRTC kernels --
# parity under it, then interleaved A/B at the config sizes and the headline
set -o pipefail
mkdir -p gpurun_out/r6y
RB_EXPERIMENTAL=1 RB_KERNARG_PRELOAD=14 timeout -k 10 400 python -u -m pytest tests/test_gpu_aa_configs.py tests/test_gpu_rnea_fd.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6y/gpu_tests_preload.log 2>&1 || exit 1
V="kernarg_preload=0 kernarg_preload=14"
timeout -k 10 200 python tools/ab_bench.py --kernel rnea --dtype f32 --batch 65536 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6y/ab_rnea32_b65536.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f32 --batch 65536 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6y/ab_fd32_b65536.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch 131072 --graph --layouts tiled --rounds 7 --steps 300 --variants $V > gpurun_out/r6y/ab_idfd64_b131072.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_bench.py --kernel rnea --dtype f64 --batch 1048576 --layouts tiled --rounds 9 --steps 100 --variants $V > gpurun_out/r6y/ab_rnea64_b1048576.log 2>&1 || exit 1
