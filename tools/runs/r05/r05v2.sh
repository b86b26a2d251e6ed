#!/bin/bash
set -o pipefail
OUT=gpurun_out/r05v2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || exit 1
grep -o "\"value\": [0-9.]*" $OUT/bench.log $OUT/bench20.log; tail -1 $OUT/gpu_tests.log; tail -2 $OUT/smoke.log
