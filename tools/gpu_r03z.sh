# round 3 (session 2): config 2 re-checks on the current build, interleaved over 3 rounds:
# st1 = one stream (default), st2 = consecutive 1M launches alternating two streams,
# o3 = the 3-waves-per-SIMD verify variant (NT_VERIFY_OCC=3)
set -o pipefail
mkdir -p gpurun_out/r03z
B="--no-sha --no-certs --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3; do
  for v in st1 st2 o3; do
    case $v in st1) E="NT_BENCH_STREAMS=1";; st2) E="NT_BENCH_STREAMS=2";; o3) E="NT_VERIFY_OCC=3";; esac
    env $E timeout -k 10 200 python -u bench.py $B > gpurun_out/r03z/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03z/${v}_r$r.log | head -1)"
  done
done
