#!/bin/bash
# Kernel-trace --stats summary of the driver's bench command on the final tree
# (the committee-sized sort LDS and the one-ballot k_ks_init included), and the
# config-2 launches under the profiler against the bench line's own kernel_ms.
set -o pipefail
OUT=gpurun_out/${1:-r06k}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run -- python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_under_rocprof.log" 2>&1 || { tail -20 $OUT/bench_under_rocprof.log; exit 1; }
DB=$(ls $OUT/stats/run_results.db $OUT/stats/*/run_results.db 2>/dev/null | head -1)
python3 tools/rocprof_summary.py $DB $OUT/rocprof_kernel_stats.csv
python3 tools/cfg2_launches.py $DB $OUT/bench_under_rocprof.log > $OUT/cfg2_launches_under_rocprof.txt
cat $OUT/cfg2_launches_under_rocprof.txt | tail -3
head -8 $OUT/rocprof_kernel_stats.csv | cut -c1-160
