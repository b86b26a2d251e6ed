# round 3 (session 2): LLVM scheduler variants (device code only) on config 2 and config 3,
# interleaved over 3 rounds: def = default, trk = -amdgpu-use-amdgpu-trackers,
# mmc = -misched=gcn-max-memory-clause
set -o pipefail
mkdir -p gpurun_out/r03af
A="--no-sha --no-ingest --no-latency --no-cpu --steps 20"
for r in 1 2 3; do
  for v in def trk mmc; do
    if [ $v = def ]; then L=narwhal-tusk_amd/lib/libntcrypto.so; else L=alt/$v/libntcrypto.so; fi
    NT_BENCH_SHARDS=0 NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03af/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.]*' gpurun_out/r03af/${v}_r$r.log | head -1) $(grep -o '"keyset": {"certs_per_s": [0-9.]*' gpurun_out/r03af/${v}_r$r.log | head -1)"
  done
done
