# round 3: single-change A/B of the verify trims (config 2 only), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/r03f
A="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 10"
for r in 1 2 3; do
  for v in alloff nocarry dblsub4 tabdbl tabdbl2 signed; do
    NTCRYPTO_LIB=alt/$v/libntcrypto.so timeout -k 10 200 python -u bench.py $A > gpurun_out/r03f/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03f/${v}_r$r.log | head -1)"
  done
done
