#!/bin/bash
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/host_pipe_probe.py > $OUT/host_pipe.json 2> $OUT/host_pipe.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/hp_trace -o run -- python3 -u tools/host_pipe_probe.py --reps 3 > $OUT/host_pipe_rocprof.json 2> $OUT/host_pipe_rocprof.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
