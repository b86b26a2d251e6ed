# round 3: rows per key-cache chunk x waves per SIMD (library built for 64 rows per chunk),
# config 3 + its 2/4/8-GPU shards, interleaved, 3 rounds.  v = cap:waves (waves 0 = the plan's choice)
set -o pipefail
mkdir -p gpurun_out/r03m
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in 8:0 32:0 64:0 64:2 32:3 16:3 48:0; do
    p=${v%:*}; w=${v#*:}
    if [ $w = 0 ]; then unset NT_KEYSET_WAVES; else export NT_KEYSET_WAVES=$w; fi
    NT_KEYSET_PER_LANE=$p NTCRYPTO_LIB=alt/ks64/libntcrypto.so timeout -k 10 300 python -u bench.py $A > gpurun_out/r03m/p${p}w${w}_r$r.log 2>&1 || exit 1
    echo "p$p w$w r$r $(python3 - gpurun_out/r03m/p${p}w${w}_r$r.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{") and '"metric"' in line:
        c = json.loads(line)["certificates"]
        print(c["keyset"]["certs_per_s"], c["keyset_one_stream"]["certs_per_s"], c["keyset"]["mismatches_vs_expected"],
              " ".join("%s:%.0f" % (k, v["certs_per_s"]) for k, v in c.get("shard_of", {}).items() if isinstance(v, dict)))
PY
)"
  done
done
