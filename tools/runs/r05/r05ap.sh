#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ap
timeout -k 10 200 python3 -u tools/host_pipe_probe.py --reps 5 > gpurun_out/r05ap/probe_plain.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05ap/tr -o run -- python3 -u tools/host_pipe_probe.py --reps 3 > gpurun_out/r05ap/probe.log 2>&1
rc=$?
grep "^{" gpurun_out/r05ap/probe_plain.log
exit $rc
