#!/bin/bash
# Interleaved A/B of two builds of libntcrypto.so on config 3 (key cache, shards,
# host entry points): bash ab_lib.sh <outdir> <name_a>=<lib_a> <name_b>=<lib_b> [rounds]
set -o pipefail
OUT=gpurun_out/$1; A=$2; B=$3; R=${4:-3}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for ab in $A $B; do
    name=${ab%%=*}; lib=${ab#*=}
    NTCRYPTO_LIB=$lib timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-sha --no-ingest --no-latency --no-cpu \
      > $OUT/${name}_$r.log 2> $OUT/${name}_$r.err || { tail -5 $OUT/${name}_$r.err; exit 1; }
    python - $OUT/${name}_$r.log "$name r$r" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
c = d["certificates"]
so = c["shard_of"]
print("%-16s cfg3 %.3f one_stream %.3f  shards %s  (M/s %s)  host_api %.3f plain %.3f  launch %.3f ms  mism %d/%s" % (
    sys.argv[2], c["value"] / 1e6, c["keyset_one_stream"]["certs_per_s"] / 1e6,
    " / ".join("%.3f" % so[k]["per_gpu_vs_1gpu"] for k in ("2", "4", "8")),
    " / ".join("%.2f" % (so[k]["certs_per_s"] / 1e6) for k in ("2", "4", "8")),
    c["host_api"]["certs_per_s"] / 1e6, c["host_api_plain"]["certs_per_s"] / 1e6,
    c["keyset"]["roofline"]["launch_ms"], c["keyset"]["mismatches_vs_expected"],
    ",".join(str(so[k]["mismatches_vs_expected"]) for k in ("2", "4", "8"))), flush=True)
PY
  done
done
