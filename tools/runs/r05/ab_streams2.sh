#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05f}
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20 --warmup 5"
NT_BENCH_STREAM_AB=1 NT_BENCH_HOST_CERTS=0 NT_BENCH_SHARDS=0 timeout -k 10 200 python -u bench.py $A > $OUT/lib.json 2> $OUT/lib.err || exit 1
