# round 3: device-ingestion chunk size A/B (config 3 as wire bytes), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03i
A="--no-sha --no-latency --no-cpu --steps 10"
for r in 1 2 3; do
  for c in 6250 12500 25000 50000; do
    NT_BENCH_SHARDS=0 NT_INGEST_CHUNK=$c timeout -k 10 300 python -u bench.py $A > gpurun_out/r03i/c${c}_r$r.log 2>&1 || exit 1
    echo "c$c r$r $(grep -o '"device_parse": {"certs_per_s": [0-9.]*' gpurun_out/r03i/c${c}_r$r.log | head -1)"
  done
done
