#!/bin/bash
# Collect PMC counters for the verify + SHA kernels in separate rocprofv3 passes
# (one counter group per pass, --kernel-trace only beside --pmc), as
# /opt/skills/guides/MI355X_MICROARCH.md §HBM / rocprofv3 prescribes.
# Usage (on the GPU box): bash tools/pmc_collect.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 1 --warmup 0 --no-cpu ${PMC_BENCH_ARGS:-}"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pass$i" -o run -- $BENCH > "$OUT/pass$i.log" 2>&1
done
echo "pmc passes done"
