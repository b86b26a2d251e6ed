set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
