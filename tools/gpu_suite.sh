# the whole GPU suite in one process (as the driver runs it), log under gpurun_out/$1/
set -o pipefail
D=gpurun_out/${1:-suite}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1
