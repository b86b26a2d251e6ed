# round 3: verify-kernel trims A/B (config 2 only), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03e
A="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 10"
for r in 1 2 3; do
  for v in default base nosigned notabdbl; do
    if [ $v = default ]; then L=narwhal-tusk_amd/lib/libntcrypto.so; else L=alt/$v/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 200 python -u bench.py $A > gpurun_out/r03e/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03e/${v}_r$r.log | head -1)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03e/parity.log 2>&1
