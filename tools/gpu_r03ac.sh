# round 3 (session 2): point-fence A/B -- the default build (verify: sched_barrier after every field
# multiply; key cache: none) vs alt/pfence (-DNT_FENCE_POINT: one after every point operation instead),
# config 2 and config 3, interleaved over 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03ac
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3; do
  for v in f pf; do
    if [ $v = pf ]; then L=alt/pfence/libntcrypto.so; else L=narwhal-tusk_amd/lib/libntcrypto.so; fi
    NT_BENCH_SHARDS=0 NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03ac/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03ac/${v}_r$r.log | head -1) $(grep -o '"keyset": {"certs_per_s": [0-9.]*' gpurun_out/r03ac/${v}_r$r.log | head -1)"
  done
done
