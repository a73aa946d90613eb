set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 500 python -u -m pytest tests/test_gpu_aa_configs.py tests/test_gpu_rnea_fd.py tests/test_gpu_multiproc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1 || exit 1
for k in "rnea_fd f64 131072" "rnea+fd f64 131072" "rnea_fd f64 1048576" "rnea+fd f64 1048576" "fd f64 1048576" "rnea_fd f32 65536" "rnea+fd f32 65536"; do
  timeout -k 10 120 rigidbody-rs_amd/bin/batch_bench $k 4000 tiled >> gpurun_out/r6b/native.log 2>&1 || exit 1
done
