# round 3: wire tests, full GPU suite, default bench, then config-2 table-latency bound experiments
set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u -m pytest tests/test_wire.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03d/wire_tests.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03d/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03d/bench.log 2>&1 || exit 1
A="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 10"
for r in 1 2; do
  for v in default xatab xcomb; do
    if [ $v = default ]; then L=narwhal-tusk_amd/lib/libntcrypto.so; else L=alt/$v/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 200 python -u bench.py $A > gpurun_out/r03d/x_${v}_r$r.log 2>&1 || exit 1
  done
done
