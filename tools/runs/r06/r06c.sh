#!/bin/bash
# Fused key-cache epilogue (verdict bits + group AND in the kernel): the key-cache
# and registry GPU tests, then NT_KEYSET_FUSE=1 (product) vs 0 (round-5 pack + group AND
# launches), interleaved three times.
set -o pipefail
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_registry.py tests/test_wire.py -x -v --timeout 300 --timeout-method thread -m gpu -k "keyset or registry or batch or ingest or device" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/runs/r06/ab_env.sh ${1:-r06c}/ab NT_KEYSET_FUSE 1 0 3
