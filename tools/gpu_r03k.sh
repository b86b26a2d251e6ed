# round 3: key-cache launch time vs rows per wave around the 8-GPU shard (12,288 rows = 6 per wave at
# 2 waves per SIMD ... 14,336 = 7 per wave), then the device-ingestion chunk-size A/B
set -o pipefail
mkdir -p gpurun_out/r03k
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2; do
  for c in 11565 12047 12528 13010 13492; do
    NT_BENCH_SHARDS=0 timeout -k 10 200 python -u bench.py $A --certs $c > gpurun_out/r03k/rows_c${c}_r$r.log 2>&1 || exit 1
    echo "c$c r$r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r03k/rows_c${c}_r$r.log | tail -1) $(grep -o '"keyset_one_stream": {"certs_per_s": [0-9.]*, "sig_verifies_per_s": [0-9.]*, "ms_per_step": [0-9.]*, "gpu_ms_per_step": [0-9.]*' gpurun_out/r03k/rows_c${c}_r$r.log | grep -o 'gpu_ms_per_step": [0-9.]*')"
  done
done
bash tools/gpu_r03i.sh
