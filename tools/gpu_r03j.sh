# round 3 final tree: full GPU suite, smoke, default bench, then the round's profiles
set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r03j/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03j/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03j/bench.log 2>&1 && \
bash tools/profile_round.sh r03
