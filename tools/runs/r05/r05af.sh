set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05af
timeout -k 10 200 python -u tools/host_pipe_probe.py --cfg3 --reps 5 > gpurun_out/r05af/cfg3.log 2>&1 &&
timeout -k 10 200 python -u tools/host_pipe_probe.py --reps 5 > gpurun_out/r05af/cfg2.log 2>&1 &&
NT_PIPE_TRACE=1 timeout -k 10 100 python -u tools/host_pipe_probe.py --cfg3 --reps 2 > gpurun_out/r05af/cfg3_trace.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "group or chunk or keyset" > gpurun_out/r05af/tests.log 2>&1
rc=$?
tail -2 gpurun_out/r05af/tests.log
tail -1 gpurun_out/r05af/cfg3.log; tail -1 gpurun_out/r05af/cfg2.log
exit $rc
