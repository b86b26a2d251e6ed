#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ay
NT_BENCH_HOST_CERTS=0 NT_BENCH_SHARDS=0 bash tools/ab_env.sh gpurun_out/r05ay 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NTCRYPTO_LIB=alt/ilp/libntcrypto.so" "NTCRYPTO_LIB=alt/memclause/libntcrypto.so"
