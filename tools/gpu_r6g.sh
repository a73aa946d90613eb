# round 6: smoke() + driver-style bench line (the driver's round-end commands) at HEAD
set -o pipefail
D=gpurun_out/r6g
mkdir -p $D
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit 1
RB_BENCH_DETAIL=$D/detail_a.json timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_a.json 2> $D/bench_a.err || exit 1
