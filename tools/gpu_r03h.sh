# round 3: verify trims, the two winners alone and combined (config 2), interleaved, 6 rounds
set -o pipefail
mkdir -p gpurun_out/r03h
A="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3 4 5 6; do
  for v in alloff nocarry tabdbl2 nc_td; do
    NTCRYPTO_LIB=alt/$v/libntcrypto.so timeout -k 10 200 python -u bench.py $A > gpurun_out/r03h/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03h/${v}_r$r.log | head -1)"
  done
done
