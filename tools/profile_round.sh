#!/bin/bash
# Profiles committed under profiles/ for a round (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of the default bench command
#   2. PMC passes (tools/pmc_collect.sh) for cfg2 verify + cfg4 SHA-512
#   3. PMC passes for the cfg3 key-cache launch
# Usage: bash tools/profile_round.sh <tag>
set -euo pipefail
TAG=${1:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run -- python3 bench.py > "$OUT/bench_under_rocprof.log" 2>&1
echo "stats done"
PMC_BENCH_ARGS="--no-certs --no-ingest --no-latency" bash tools/pmc_collect.sh "$OUT/pmc"
python3 tools/pmc_summarize.py "$OUT/pmc" "$OUT/pmc_verify_sha.json" "cfg2 verify + cfg4 SHA-512" > /dev/null
NT_BENCH_SHARDS=0 PMC_BENCH_ARGS="--no-sha --no-ingest --no-latency --sigs 65536" bash tools/pmc_collect.sh "$OUT/pmc_keyset"
python3 tools/pmc_summarize.py "$OUT/pmc_keyset" "$OUT/pmc_keyset.json" "cfg3 key-cache launch" > /dev/null
echo "pmc done"
