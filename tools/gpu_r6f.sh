# round 6: driver-style bench lines (x2) + the rollout launcher test + near-singular FD (printed K)
set -o pipefail
D=gpurun_out/r6f
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_inputs.py "tests/test_gpu_domain.py::test_fd64_near_singular_floating_base" -v -s --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
for r in a b; do
  RB_BENCH_DETAIL=$D/detail_$r.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_$r.json 2> $D/bench_$r.err || exit 1
done
