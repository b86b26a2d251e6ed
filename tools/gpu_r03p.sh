# round 3 (session 2): baseline of the restored tree -- full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations 10 > gpurun_out/r03p/tests.log 2>&1 && \
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03p/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03p/bench.log 2>&1
