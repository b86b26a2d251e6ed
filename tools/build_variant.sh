#!/bin/bash
# Build libntcrypto.so with extra compile flags into alt/<name>/ (git-ignored,
# travels to the GPU box) for in-session A/B runs: NTCRYPTO_LIB=alt/<name>/libntcrypto.so
# Usage: bash tools/build_variant.sh <name> "<extra compile flags>"
set -euo pipefail
NAME=$1; EXTRA=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/narwhal-tusk_amd" -j8 B="../alt/$NAME/build" L="../alt/$NAME" EXTRA="$EXTRA" "../alt/$NAME/libntcrypto.so"
rm -rf "$ROOT/alt/$NAME/build"
echo "$ROOT/alt/$NAME/libntcrypto.so"
