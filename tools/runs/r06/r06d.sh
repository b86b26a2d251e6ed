#!/bin/bash
# Validation of the round-6 tree: the driver's GPU tests, smoke, the driver's
# bench command, the default bench, and a full-size two-rank rehearsal on one GPU.
set -o pipefail
OUT=gpurun_out/${1:-r06d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 1; }
python tools/bench_brief.py $OUT/bench20.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/bench_brief.py $OUT/bench.log | head -3
NT_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > $OUT/bench_2ranks.log 2> $OUT/bench_2ranks.err || { tail -30 $OUT/bench_2ranks.err; exit 1; }
python tools/bench_brief.py $OUT/bench_2ranks.log | head -6
