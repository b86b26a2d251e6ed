# round 3 (session 2): full GPU suite + smoke of the tree (streamed key-cache rows, padded / unrolled
# key sort, variable-time binary-GCD inversion), then config 3 + its 2/4/8-GPU shards interleaved over
# 3 rounds: new = the tree, so = round-2 key sort (alt/sortold), fi = Fermat inversion (alt/invfermat),
# n3 = the tree at 3 waves per SIMD
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations 10 > gpurun_out/r03t/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t/smoke.log 2>&1 || exit 1
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in new so fi n3; do
    W=""; L=narwhal-tusk_amd/lib/libntcrypto.so
    case $v in so) L=alt/sortold/libntcrypto.so;; fi) L=alt/invfermat/libntcrypto.so;; n3) W=3;; esac
    NT_KEYSET_WAVES=$W NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03t/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(python3 - gpurun_out/r03t/${v}_r$r.log <<'PY'
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
