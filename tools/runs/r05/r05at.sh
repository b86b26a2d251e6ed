#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05at
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "keyset or group" > gpurun_out/r05at/tests.log 2>&1 || { tail -30 gpurun_out/r05at/tests.log; exit 1; }
tail -1 gpurun_out/r05at/tests.log
NT_BENCH_HOST_CERTS=0 bash tools/ab_env.sh gpurun_out/r05at 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NT_SORT_LDS_FULL=1"
NT_BENCH_HOST_CERTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05at/tr -o run -- python3 bench.py --no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5 > gpurun_out/r05at/bench_tr.log 2>&1
