# round 6: fused-pair tests (host-pointer form), fp32 fused vs two calls at 2^20, 12-link chain
set -o pipefail
D=gpurun_out/r6k
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_rnea_fd.py -x -v --timeout 200 --timeout-method thread > $D/tests.log 2>&1 || exit 1
for k in "rnea_fd f32 1048576" "rnea+fd f32 1048576" "rnea f32 1048576" "fd f32 1048576"; do
  timeout -k 10 120 rigidbody-rs_amd/bin/batch_bench $k 3000 tiled >> $D/native.log 2>&1 || exit 1
done
