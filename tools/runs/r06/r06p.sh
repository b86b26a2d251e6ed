#!/bin/bash
# Round-6 profiles (run on the GPU box): the kernel-trace --stats summary of the
# driver's bench command, the PMC passes (clock probe included, so the probe's
# in-kernel clock and the kernels' GRBM clocks come from the same process), and
# a kernel trace of the config-3 shard steps.
set -euo pipefail
TAG=${1:-r06p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run -- python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_under_rocprof.log" 2>&1
echo "stats done"
PMC_BENCH_ARGS="--no-certs --no-ingest --no-latency" bash tools/pmc_collect.sh "$OUT/pmc"
python3 tools/pmc_summarize.py "$OUT/pmc" "$OUT/pmc_verify_sha.json" "cfg2 verify + cfg4 SHA-512 + clock probe" > /dev/null
NT_BENCH_SHARDS=0 NT_BENCH_HOST_CERTS=0 PMC_BENCH_ARGS="--no-sha --no-ingest --no-latency --sigs 65536" bash tools/pmc_collect.sh "$OUT/pmc_keyset"
python3 tools/pmc_summarize.py "$OUT/pmc_keyset" "$OUT/pmc_keyset.json" "cfg3 key-cache launch + clock probe" > /dev/null
echo "pmc done"
NT_BENCH_HOST_CERTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- python3 bench.py --no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5 > "$OUT/bench_trace.log" 2>&1
echo "trace done"
