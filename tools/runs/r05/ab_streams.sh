#!/bin/bash
# session A/B: config-3 steps on library vs torch streams, interleaved
set -o pipefail
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20 --warmup 5"
for r in 1 2; do
  NT_BENCH_STREAM_AB=1 NT_BENCH_LIB_STREAMS=1 timeout -k 10 200 python -u bench.py $A > $OUT/lib_$r.json 2> $OUT/lib_$r.err || exit 1
  NT_BENCH_LIB_STREAMS=0 timeout -k 10 200 python -u bench.py $A > $OUT/torch_$r.json 2> $OUT/torch_$r.err || exit 1
done
