# round 3, first GPU pass: parity tests, smoke, default bench, then key-cache wave A/B (certificates only)
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03a/bench.log 2>&1 && \
for w in 2 3; do
  NT_KEYSET_WAVES=$w timeout -k 10 200 python -u bench.py --no-sha --no-ingest --no-latency --no-cpu --steps 5 > gpurun_out/r03a/certs_w$w.log 2>&1 || exit 1
done
