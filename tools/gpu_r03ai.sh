# round 3 (session 2): LLVM scheduler of k_misc.hip (config 4's k_sha512_pipe consumer wave runs alone
# on its SIMD, so its instruction order is its latency), interleaved over 3 rounds:
# def = default, milp = -misched=gcn-max-ilp, mmmc = -misched=gcn-max-memory-clause
set -o pipefail
mkdir -p gpurun_out/r03ai
A="--no-certs --no-ingest --no-latency --no-cpu --sigs 65536 --steps 5"
for r in 1 2 3; do
  for v in def milp mmmc; do
    if [ $v = def ]; then L=narwhal-tusk_amd/lib/libntcrypto.so; else L=alt/$v/libntcrypto.so; fi
    NTCRYPTO_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/r03ai/${v}_r$r.log 2>&1 || exit 1
    echo "$v r$r $(python3 - gpurun_out/r03ai/${v}_r$r.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{") and '"metric"' in line:
        s = json.loads(line)["sha512"]
        print(s["value"], s["kernel_ms"])
PY
)"
  done
done
