# round 3 (session 2): streamed key-cache rows -- key-cache / certificate GPU tests with the new
# default, then config 3 + its 2/4/8-GPU shards, interleaved A/B over 3 rounds:
# s2 = streamed rows at 2 waves/SIMD (default), s3 = streamed at 3, c = chunked plan (NT_KEYSET_STREAM=0)
set -o pipefail
mkdir -p gpurun_out/r03q
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_wire.py tests/test_cpp_mirror.py -x -v -m gpu -k "keyset or cert or ingest or wire or groups" --timeout 600 --timeout-method thread --durations 10 > gpurun_out/r03q/tests.log 2>&1 || exit 1
A="--no-sha --no-ingest --no-latency --no-cpu --sigs 65536 --steps 10"
for r in 1 2 3; do
  for v in s2 c s3; do
    case $v in s2) E="NT_KEYSET_STREAM=1";; s3) E="NT_KEYSET_STREAM=1 NT_KEYSET_WAVES=3";; c) E="NT_KEYSET_STREAM=0";; esac
    env $E timeout -k 10 300 python -u bench.py $A > gpurun_out/r03q/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(python3 - gpurun_out/r03q/${v}_r$r.log <<'PY'
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
# config 2: pre-scaled operands shared in the point conversions (default) vs not (alt/ps0)
B="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3; do
  for v in ps1 ps0; do
    if [ $v = ps0 ]; then L=alt/ps0/libntcrypto.so; else L=narwhal-tusk_amd/lib/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/r03q/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03q/${v}_r$r.log | head -1)"
  done
done
