# round 3 (session 2): LLVM scheduler of the key-cache kernels (device code), config 3 + shards,
# interleaved over 3 rounds: def = default, kilp = -misched=gcn-max-ilp, kocc = -misched=gcn-max-occupancy
set -o pipefail
mkdir -p gpurun_out/r03ah
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in def kilp kocc; do
    if [ $v = def ]; then L=narwhal-tusk_amd/lib/libntcrypto.so; else L=alt/$v/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03ah/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(python3 - gpurun_out/r03ah/${v}_r$r.log <<'PY'
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
