#!/bin/bash
# Handoff of every wave's last batch to the last wave of its workgroup
# (-DNT_KS_HANDOFF=1, alt/handoff): the key-cache / registry / ingestion GPU
# tests against that build, then config 3 and its shards interleaved with the
# product build three times.  The variant: git apply tools/experiments/ks_handoff.patch &&
# bash tools/build_variant.sh handoff "-DNT_KS_HANDOFF=1" && git checkout narwhal-tusk_amd/csrc/k_keyset.inc
set -o pipefail
OUT=gpurun_out/${1:-r06l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__)" || exit 1
NTCRYPTO_LIB=alt/handoff/libntcrypto.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_registry.py tests/test_gpu_fullsize.py tests/test_wire.py tests/test_gpu_memory.py -x -q -m gpu --timeout 300 --timeout-method thread -k "keyset or registry or cfg3 or batch or ingest or budget" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/runs/r06/ab_lib.sh ${1:-r06l}/ab product=narwhal-tusk_amd/lib/libntcrypto.so handoff=alt/handoff/libntcrypto.so 3
