#!/bin/bash
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 1
