# round 3: key-cache plan scan on config 3 (1 GPU): chunks per wave k = 1..6 at 2 and 3 waves per
# SIMD (cap = rows per chunk that yields k; library built for 64), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03n
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in 52:2 26:2 18:2 13:2 11:2 9:2 35:3 18:3 12:3 9:3 7:3; do
    p=${v%:*}; w=${v#*:}
    NT_BENCH_SHARDS=0 NT_KEYSET_WAVES=$w NT_KEYSET_PER_LANE=$p NTCRYPTO_LIB=alt/ks64/libntcrypto.so timeout -k 10 300 python -u bench.py $A > gpurun_out/r03n/p${p}w${w}_r$r.log 2>&1 || exit 1
    echo "p$p w$w r$r $(python3 - gpurun_out/r03n/p${p}w${w}_r$r.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{") and '"metric"' in line:
        c = json.loads(line)["certificates"]
        print(c["keyset"]["certs_per_s"], c["keyset_one_stream"]["certs_per_s"], c["keyset"]["roofline"]["launch_ms"],
              c["keyset"]["mismatches_vs_expected"])
PY
)"
  done
done
