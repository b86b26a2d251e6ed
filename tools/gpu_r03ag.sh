# round 3 (session 2): final validation of the tree after the verify kernels moved to the memory-clause scheduler (and the
# key-cache fence and sort changes) -- full GPU suite, smoke, two default bench runs
set -o pipefail
mkdir -p gpurun_out/r03ag
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations 10 > gpurun_out/r03ag/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ag/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03ag/bench1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03ag/bench2.log 2>&1
