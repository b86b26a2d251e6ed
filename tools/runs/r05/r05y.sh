#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05y
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05y/gpu_tests.log 2>&1 || exit 1
NT_BENCH_HOST_CERTS=0 bash tools/ab_env.sh gpurun_out/r05y 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NT_KEYSET_COMB_BITS=20"
