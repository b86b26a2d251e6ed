#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aq
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunk or host or group or keyset" > gpurun_out/r05aq/tests.log 2>&1 || { tail -30 gpurun_out/r05aq/tests.log; exit 1; }
tail -1 gpurun_out/r05aq/tests.log
for r in 1 2; do
for v in 2 1; do
NT_COPY_STREAMS=$v timeout -k 10 120 python3 -u tools/host_pipe_probe.py --reps 5 > gpurun_out/r05aq/cfg2_s${v}_r$r.log 2>&1 || exit 1
NT_COPY_STREAMS=$v timeout -k 10 120 python3 -u tools/host_pipe_probe.py --cfg3 --reps 5 > gpurun_out/r05aq/cfg3_s${v}_r$r.log 2>&1 || exit 1
echo "streams $v round $r: $(grep '^{' gpurun_out/r05aq/cfg2_s${v}_r$r.log | cut -c1-150)"
echo "streams $v round $r: $(grep '^{' gpurun_out/r05aq/cfg3_s${v}_r$r.log | cut -c1-200)"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05aq/tr -o run -- python3 -u tools/host_pipe_probe.py --reps 3 > gpurun_out/r05aq/probe_tr.log 2>&1
