#!/bin/bash
# Final-tree validation (the driver's round-end sequence): the whole GPU suite,
# smoke, the driver's bench command and the default bench.  torch is imported
# once first (the first import on a fresh box pages the image in); a heartbeat
# file marks progress while a long step runs (each step keeps its own limit).
set -o pipefail
OUT=gpurun_out/${1:-r06j}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__)" || exit 1
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread --durations=5 > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -8 $OUT/gpu_tests.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 1; }
python tools/bench_brief.py $OUT/bench20.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/bench_brief.py $OUT/bench.log | head -4
