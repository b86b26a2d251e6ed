# round 3 (session 2): last validation of the committed tree (same sources as r03ag plus the empty
# MISC_SCHED hook) -- full GPU suite, smoke, two default bench runs
set -o pipefail
mkdir -p gpurun_out/r03aj
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations 10 > gpurun_out/r03aj/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aj/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03aj/bench1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03aj/bench2.log 2>&1
