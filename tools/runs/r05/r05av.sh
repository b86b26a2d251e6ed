#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05av
for r in 1 2; do
for v in 4 3 2; do
NT_PIPE_MID=$v timeout -k 10 120 python3 -u tools/host_pipe_probe.py --cfg3 --reps 5 > gpurun_out/r05av/cfg3_${v}_r$r.log 2>&1 || exit 1
echo "mid $v r$r: $(grep '^{' gpurun_out/r05av/cfg3_${v}_r$r.log | cut -c1-150)"
done; done
