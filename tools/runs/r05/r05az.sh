#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05az
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "group or keyset or chunk" > gpurun_out/r05az/tests.log 2>&1 || { tail -30 gpurun_out/r05az/tests.log; exit 1; }
tail -1 gpurun_out/r05az/tests.log
for r in 1 2; do
for v in new gather; do
if [ $v = gather ]; then export NT_GROUPS_GATHER=1; else unset NT_GROUPS_GATHER; fi
timeout -k 10 120 python3 -u tools/host_pipe_probe.py --cfg3 --reps 5 > gpurun_out/r05az/cfg3_${v}_r$r.log 2>&1 || exit 1
echo "$v r$r: $(grep '^{' gpurun_out/r05az/cfg3_${v}_r$r.log | cut -c60-330)"
done; done
