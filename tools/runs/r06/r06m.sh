#!/bin/bash
# Registry chunks copy their signatures before waiting for the chunk's key
# lookups (the product build) vs the lookups-first order (alt/base: the tree
# before the change, tools/build_variant.sh base ""): the registry / groups GPU
# tests, then config 3's host entry points interleaved three times.
set -o pipefail
OUT=gpurun_out/${1:-r06m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__)" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_registry.py tests/test_gpu_parity.py tests/test_gpu_sharding.py -x -q -m gpu --timeout 300 --timeout-method thread -k "registry or groups or batch or concurrent" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
bash tools/runs/r06/ab_lib.sh ${1:-r06m}/ab base=alt/base/libntcrypto.so sigsfirst=narwhal-tusk_amd/lib/libntcrypto.so 3
