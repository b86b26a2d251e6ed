# round 3: key-cache plan with chunks up to 64 rows (default): key-cache GPU tests, the full-size
# tests, the default bench, then the device-ingestion chunk-size A/B
set -o pipefail
mkdir -p gpurun_out/r03o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py tests/test_gpu_fullsize.py -x -v -m gpu -k "keyset or wire or ingest or cert or fullsize" --timeout 600 --timeout-method thread --durations 15 > gpurun_out/r03o/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03o/bench.log 2>&1 && \
bash tools/gpu_r03i.sh
