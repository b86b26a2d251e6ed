#!/bin/bash
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20 --warmup 5"
NT_BENCH_STREAM_AB=1 timeout -k 10 200 python -u bench.py $A > $OUT/lib.json 2> $OUT/lib.err || exit 1
NT_BENCH_LIB_STREAMS=0 NT_BENCH_SHARDS=1 timeout -k 10 200 python -u bench.py $A > $OUT/torch.json 2> $OUT/torch.err || exit 1
timeout -k 10 120 python -u tools/host_pipe_probe.py > $OUT/host_pipe.json 2> $OUT/host_pipe.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/hp_trace -o run -- python3 -u tools/host_pipe_probe.py --reps 3 > $OUT/host_pipe_rocprof.json 2> $OUT/host_pipe_rocprof.err || exit 1
