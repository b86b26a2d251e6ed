#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 20 --warmup 5"
NT_BENCH_STREAM_AB=1 NT_BENCH_HOST_CERTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/lib -o run -- python3 -u bench.py $A > $OUT/lib.json 2> $OUT/lib.err || exit 1
NT_BENCH_LIB_STREAMS=0 NT_BENCH_HOST_CERTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/torch -o run -- python3 -u bench.py $A > $OUT/torch.json 2> $OUT/torch.err || exit 1
