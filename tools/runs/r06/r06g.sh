#!/bin/bash
# Committee-sized sort LDS + one-ballot group-word init: the whole GPU suite
# (with the registry concurrency test), smoke, the driver's bench command, and a
# kernel trace of the config-3 shard steps (tools/shard_steps.py).
# torch is imported once first (the first import on a fresh box pages the image
# in for 1-2 minutes with nothing to print); a heartbeat file marks progress
# while a long test runs (each step keeps its own time limit).
set -o pipefail
OUT=gpurun_out/${1:-r06g}
mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__)" || exit 1
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread --durations=12 > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -16 $OUT/gpu_tests.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 1; }
python tools/bench_brief.py $OUT/bench20.log
NT_BENCH_HOST_CERTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- python3 bench.py --no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5 > "$OUT/bench_trace.log" 2>&1 || { tail -20 $OUT/bench_trace.log; exit 1; }
python tools/shard_steps.py $(ls $OUT/tr/*/run_kernel_trace.csv $OUT/tr/run_kernel_trace.csv 2>/dev/null | head -1) 20 6 > $OUT/shard8_trace.txt
head -8 $OUT/shard8_trace.txt
