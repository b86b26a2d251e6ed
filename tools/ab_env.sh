#!/bin/bash
# A/B of run-time variants within ONE GPU session (box-to-box clock differences
# are several percent, so variants are interleaved and repeated).
# Usage: bash tools/ab_env.sh <outdir> <rounds> "<bench args>" "VAR=a VAR2=b" "VAR=c" ...
set -euo pipefail
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python3 bench.py $ARGS > "$OUT/v${i}_r${r}.log" 2>&1
    echo "$v round $r: $(grep -o '"value": [0-9.]*' "$OUT/v${i}_r${r}.log" | head -1)"
  done
done
