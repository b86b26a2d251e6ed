#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ar
for r in 1 2; do
for v in 131072 262144 393216; do
NT_PIPE_ROUND=$v timeout -k 10 120 python3 -u tools/host_pipe_probe.py --reps 5 > gpurun_out/r05ar/cfg2_${v}_r$r.log 2>&1 || exit 1
echo "round $v r$r: $(grep '^{' gpurun_out/r05ar/cfg2_${v}_r$r.log | cut -c1-170)"
done; done
