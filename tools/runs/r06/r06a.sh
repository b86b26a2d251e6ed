#!/bin/bash
# First GPU pass of round 6: the key registry's GPU tests, then the whole GPU
# suite, smoke and the default bench.
set -o pipefail
OUT=gpurun_out/${1:-r06a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_registry.py tests/test_small_call.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_registry.log 2>&1 || { tail -40 $OUT/gpu_registry.log; exit 1; }
tail -3 $OUT/gpu_registry.log
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench20.log 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 1; }
python tools/bench_brief.py $OUT/bench20.log
