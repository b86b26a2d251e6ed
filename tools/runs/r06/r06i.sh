#!/bin/bash
# Address translation on the key-cache launch: UTCL1 counters of the config-3
# launch with the driver's placement and with the comb tables in physically
# contiguous VRAM (NT_TABLE_ALLOC=contig), then the two interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r06i}
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-sha --no-ingest --no-latency --sigs 65536"
CTR="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"
for v in default contig; do
  NT_TABLE_ALLOC=$v NT_REG_TRACE=1 NT_BENCH_SHARDS=0 NT_BENCH_HOST_CERTS=0 timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d "$OUT/tlb_$v" -o run -- $BENCH > "$OUT/tlb_$v.log" 2>&1 || { tail -20 $OUT/tlb_$v.log; exit 1; }
  echo "== $v"; grep "\[alloc\]" $OUT/tlb_$v.log | sort | uniq -c | head -5
  python3 tools/pmc_kernel.py $OUT/tlb_$v/run_counter_collection.csv keyset 3
  python3 tools/pmc_kernel.py $OUT/tlb_$v/run_counter_collection.csv k_ed25519_verify 2
done
bash tools/runs/r06/ab_env.sh ${1:-r06i}/ab NT_TABLE_ALLOC default contig 2
