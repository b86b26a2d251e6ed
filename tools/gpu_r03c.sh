# round 3: device wire ingestion -- wire tests first, then the full GPU suite and the default bench
set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_wire.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03c/wire_tests.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03c/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03c/bench.log 2>&1
