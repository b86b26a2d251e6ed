#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05an
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "keyset" > gpurun_out/r05an/tests.log 2>&1 || { tail -30 gpurun_out/r05an/tests.log; exit 1; }
tail -2 gpurun_out/r05an/tests.log
NT_BENCH_HOST_CERTS=0 bash tools/ab_env.sh gpurun_out/r05an 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NTCRYPTO_LIB=alt/noexit/libntcrypto.so"
