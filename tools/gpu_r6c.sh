# round 6: fused pair tests, then graph A/B of the wave split (fp64 FD and the fused pair)
set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 500 python -u -m pytest tests/test_gpu_aa_configs.py tests/test_gpu_rnea_fd.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6c/tests.log 2>&1 || exit 1
for B in 65536 131072 262144; do
  timeout -k 10 200 python tools/ab_bench.py --kernel fd --dtype f64 --batch $B --graph --layouts tiled --rounds 5 --steps 400 --variants pack=-1 pack=5 > gpurun_out/r6c/ab_fd64_b$B.log 2>&1 || exit 1
  timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f64 --batch $B --graph --layouts tiled --rounds 5 --steps 400 --variants pack=1 pack=5 > gpurun_out/r6c/ab_idfd64_b$B.log 2>&1 || exit 1
done
for B in 65536 131072; do
  timeout -k 10 200 python tools/ab_bench.py --kernel rnea_fd --dtype f32 --batch $B --graph --layouts tiled --rounds 5 --steps 400 --variants pack=1 pack=5 > gpurun_out/r6c/ab_idfd32_b$B.log 2>&1 || exit 1
done
