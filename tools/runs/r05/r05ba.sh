#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ba
NT_BENCH_HOST_CERTS=0 bash tools/ab_env.sh gpurun_out/r05ba 3 "--no-ingest --no-latency --no-cpu --no-sha --sigs 65536 --steps 20 --warmup 5" "NT_X=base" "NT_KEYSET_WAVES=2"
