#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ax
NT_BENCH_DEVICE=0 timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r05ax/bench_2ranks.log 2>&1
rc=$?
grep -o '"value": [0-9.]*' gpurun_out/r05ax/bench_2ranks.log | head -3
tail -3 gpurun_out/r05ax/bench_2ranks.log | cut -c1-300
exit $rc
