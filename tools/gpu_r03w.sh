# round 3 (session 2): device-ingestion chunk size with the streamed key-cache kernel
# (config 3 as wire bytes, PCIe-inclusive), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03w
A="--no-sha --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for c in 3125 4096 6250 9000 12500 25000; do
    NT_BENCH_SHARDS=0 NT_INGEST_CHUNK=$c timeout -k 10 300 python -u bench.py $A > gpurun_out/r03w/c${c}_r$r.log 2>&1 || exit 1
    echo "c$c r$r $(grep -o '"device_parse": {"certs_per_s": [0-9.]*' gpurun_out/r03w/c${c}_r$r.log | head -1)"
  done
done
