#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05as
NT_BENCH_HOST_CERTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05as/tr -o run -- python3 bench.py --no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5 > gpurun_out/r05as/bench.log 2>&1
