# round 6: headline form A/B with more rounds (policy = sequential pair + 75% tail vs one per lane)
set -o pipefail
mkdir -p gpurun_out/r6i
for rep in 1 2; do
timeout -k 10 300 python tools/ab_bench.py --kernel rnea --dtype f64 --layouts tiled --rounds 12 --steps 300 \
  --variants pack=-1 pack=1 seq_tail=50 > gpurun_out/r6i/ab_rnea64_forms_$rep.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_bench.py --kernel rnea --dtype f64 --layouts tiled --rounds 12 --steps 300 \
  --variants pack=1 pack=-1 seq_tail=50 > gpurun_out/r6i/ab_rnea64_forms_rev_$rep.log 2>&1 || exit 1
done
