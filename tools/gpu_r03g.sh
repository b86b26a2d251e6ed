# round 3: combined verify trims, interleaved A/B over config 2 and config 3, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03g
A="--no-sha --no-ingest --no-latency --no-cpu --steps 10"
for r in 1 2 3; do
  for v in alloff nocarry tabdbl2 nc_td nc_td_ds; do
    NT_BENCH_SHARDS=0 NTCRYPTO_LIB=alt/$v/libntcrypto.so timeout -k 10 300 python -u bench.py $A > gpurun_out/r03g/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03g/${v}_r$r.log | head -1) $(grep -o '"certs_per_s": [0-9.]*' gpurun_out/r03g/${v}_r$r.log | head -2 | tr '\n' ' ')"
  done
done
