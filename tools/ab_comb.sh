#!/bin/bash
# Config-3 key-cache comb width A/B (16 / 18 / 20-bit combs of -A), interleaved
# within one GPU session, plus PMC passes (issue share, traffic per launch) for
# the mixed-mode key-cache launch at each width.
set -euo pipefail
OUT=${1:-gpurun_out/ab_comb}
mkdir -p "$OUT"
bash tools/ab_env.sh "$OUT" 3 "--no-sha --no-cpu --no-ingest --no-latency --sigs 65536 --steps 5" \
  "NT_KEYSET_COMB_BITS=16" "NT_KEYSET_COMB_BITS=18" "NT_KEYSET_COMB_BITS=20"
for b in 18 20; do
  NT_KEYSET_COMB_BITS=$b PMC_BENCH_ARGS="--no-sha --no-ingest --no-latency --sigs 65536" \
    bash tools/pmc_collect.sh "$OUT/pmc_w$b"
  python3 tools/pmc_summarize.py "$OUT/pmc_w$b" "$OUT/pmc_keyset_w$b.json" "keyset comb $b bits" > /dev/null
done
echo "ab_comb done"
