# the driver's round-end GPU commands at HEAD, in order: pytest -m gpu, smoke(), bench.py (N = 1)
set -o pipefail
D=gpurun_out/${1:-final}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
RB_BENCH_DETAIL=$D/bench_detail.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || exit 1
