# round 3 (session 2): full GPU suite + smoke of the tree with streamed key-cache rows and the
# padded / unrolled key sort; sort A/B (new vs alt/sortold) on config 3 + shards, 3 rounds; default bench
set -o pipefail
mkdir -p gpurun_out/r03r
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations 10 > gpurun_out/r03r/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r/smoke.log 2>&1 || exit 1
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then L=alt/sortold/libntcrypto.so; else L=narwhal-tusk_amd/lib/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03r/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(python3 - gpurun_out/r03r/${v}_r$r.log <<'PY'
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
timeout -k 10 300 python -u bench.py > gpurun_out/r03r/bench.log 2>&1
