#!/bin/bash
# Key-comb width A/B: the driver's bench command with the
# committee key combs at 21 bits (reduced scalars) and 20 bits, interleaved
# twice on one box.  Run on two fresh boxes; compare certs_per_s.
set -o pipefail
OUT=gpurun_out/${1:-r06w}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for w in 21 20; do
    NT_KEYSET_COMB_BITS=$w timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu \
      > $OUT/bench_w${w}_${rep}.log 2> $OUT/bench_w${w}_${rep}.err || exit 1
    python - $OUT/bench_w${w}_${rep}.log $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["certificates"]
print("w%s cfg2 %.2f M/s  cfg3 %.3f M certs/s  one_stream %.3f  shards %s  host_api %.3f" % (
    sys.argv[2], d["value"] / 1e6, c["value"] / 1e6, c["keyset_one_stream"]["certs_per_s"] / 1e6,
    " / ".join("%.3f" % c["shard_of"][k]["per_gpu_vs_1gpu"] for k in ("2", "4", "8")),
    c["host_api"]["certs_per_s"] / 1e6), flush=True)
PY
  done
done
