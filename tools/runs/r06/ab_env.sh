#!/bin/bash
# Interleaved A/B of one environment knob on config 3 (key cache, shards, host
# entry points): bash ab_env.sh <outdir> <VAR> <value_a> <value_b> [rounds]
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; A=$3; B=$4; R=${5:-3}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-sha --no-ingest --no-latency --no-cpu \
      > $OUT/${VAR}_${v}_$r.log 2> $OUT/${VAR}_${v}_$r.err || { tail -5 $OUT/${VAR}_${v}_$r.err; exit 1; }
    python - $OUT/${VAR}_${v}_$r.log "$VAR=$v r$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["certificates"]
so = c["shard_of"]
print("%-22s cfg3 %.3f one_stream %.3f  shards %s  (M/s %s)  host_api %.3f plain %.3f  launch %.3f ms  mism %d" % (
    sys.argv[2], c["value"] / 1e6, c["keyset_one_stream"]["certs_per_s"] / 1e6,
    " / ".join("%.3f" % so[k]["per_gpu_vs_1gpu"] for k in ("2", "4", "8")),
    " / ".join("%.2f" % (so[k]["certs_per_s"] / 1e6) for k in ("2", "4", "8")),
    c["host_api"]["certs_per_s"] / 1e6, c["host_api_plain"]["certs_per_s"] / 1e6,
    c["keyset"]["roofline"]["launch_ms"], c["keyset"]["mismatches_vs_expected"]), flush=True)
PY
  done
done
