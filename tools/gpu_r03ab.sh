# round 3 (session 2): scheduling-fence A/B -- the default build (sched_barrier after every field
# multiply) vs alt/nofence (-DNT_NO_MUL_FENCE), config 2 and config 3, interleaved over 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03ab
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3; do
  for v in f nf; do
    if [ $v = nf ]; then L=alt/nofence/libntcrypto.so; else L=narwhal-tusk_amd/lib/libntcrypto.so; fi
    NT_BENCH_SHARDS=0 NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03ab/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03ab/${v}_r$r.log | head -1) $(grep -o '"keyset": {"certs_per_s": [0-9.]*' gpurun_out/r03ab/${v}_r$r.log | head -1)"
  done
done
