#!/bin/bash
# Build libntcrypto.so with extra compile flags into alt/<name>/ (git-ignored,
# travels to the GPU box) for in-session A/B runs: NTCRYPTO_LIB=alt/<name>/libntcrypto.so
# Usage: bash tools/build_variant.sh <name> "<extra hipcc flags>"
set -euo pipefail
NAME=$1; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/narwhal-tusk_amd/csrc
OUT=$ROOT/alt/$NAME
mkdir -p "$OUT/obj"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $EXTRA"
pids=()
for tu in k_misc k_verify_strict k_verify_cofactorless k_keyset_strict_w20 k_keyset_strict_w16 \
          k_keyset_cofactorless_w20 k_keyset_cofactorless_w16 k_keyset_mixed_w20 k_keyset_mixed_w16; do
  /opt/rocm/bin/hipcc $FLAGS -c -x hip "$SRC/$tu.hip" -o "$OUT/obj/$tu.o" & pids+=($!)
done
/opt/rocm/bin/hipcc $FLAGS -c -x hip "$SRC/ntcrypto.cpp" -o "$OUT/obj/ntcrypto.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$OUT"/obj/*.o -o "$OUT/libntcrypto.so"
rm -rf "$OUT/obj"
echo "$OUT/libntcrypto.so"
