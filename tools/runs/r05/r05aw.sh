#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aw
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sha512" > gpurun_out/r05aw/tests.log 2>&1
rc=$?
tail -8 gpurun_out/r05aw/tests.log
exit $rc
