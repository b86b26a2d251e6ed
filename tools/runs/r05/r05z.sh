#!/bin/bash
set -o pipefail
export TMPDIR=/tmp NT_BENCH_HOST_CERTS=0
bash tools/ab_env.sh gpurun_out/r05z 3 "--no-ingest --no-latency --no-cpu --no-sha --steps 20 --warmup 5" "NT_X=base" "NTCRYPTO_LIB=alt/b26/libntcrypto.so"
