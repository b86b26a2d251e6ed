#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ag
NT_BENCH_HOST_CERTS=0 bash tools/ab_env.sh gpurun_out/r05ag 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NTCRYPTO_LIB=alt/noinv/libntcrypto.so"
