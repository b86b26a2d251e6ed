# round 3 (session 2): rocprof kernel stats of config 3's one-GPU step (100k certificates) and of the
# 8-GPU shard's step (12.5k certificates) run alone on one GPU, to attribute the shard's per-GPU loss
set -o pipefail
mkdir -p gpurun_out/r03u
export TMPDIR=/tmp
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for c in 100000 12500; do
  NT_BENCH_SHARDS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03u/c$c -o run -- python3 bench.py $A --certs $c > gpurun_out/r03u/c$c.log 2>&1 || exit 1
done
for c in 100000 12500; do
  db=$(find gpurun_out/r03u/c$c -name "*.db" | head -n 1)
  python3 tools/rocprof_summary.py "$db" gpurun_out/r03u/stats_c$c.csv
done
