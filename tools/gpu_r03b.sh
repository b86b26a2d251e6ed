# round 3: config-3 shard profile (kernel trace) + key-sort A/B at the shard sizes
set -o pipefail
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/prof -o run -- python3 bench.py --no-sha --no-ingest --no-latency --no-cpu --sigs 65536 > gpurun_out/r03b/bench_prof.log 2>&1 || exit 1
for r in 1 2; do
  for s in 1 0; do
    NT_KEYSET_SORT=$s timeout -k 10 200 python -u bench.py --no-sha --no-ingest --no-latency --no-cpu --sigs 65536 > gpurun_out/r03b/sort${s}_r$r.log 2>&1 || exit 1
  done
done
