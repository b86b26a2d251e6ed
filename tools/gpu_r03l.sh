# round 3: rows per key-cache chunk (one inversion each) under the persistent plan: caps 8..32
# (NT_KEYSET_PER_LANE, library built for 32), config 3 + its 2/4/8-GPU shards, interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03l
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for p in 8 12 16 24 32; do
    NT_KEYSET_PER_LANE=$p NTCRYPTO_LIB=alt/ks32/libntcrypto.so timeout -k 10 300 python -u bench.py $A > gpurun_out/r03l/p${p}_r$r.log 2>&1 || exit 1
    echo "p$p r$r $(python3 - gpurun_out/r03l/p${p}_r$r.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{") and '"metric"' in line:
        c = json.loads(line)["certificates"]
        print(c["keyset"]["certs_per_s"], c["keyset_one_stream"]["certs_per_s"], c["keyset"]["mismatches_vs_expected"],
              " ".join("%s:%.3f" % (k, v["per_gpu_vs_1gpu"]) for k, v in c.get("shard_of", {}).items() if isinstance(v, dict)))
PY
)"
  done
done
