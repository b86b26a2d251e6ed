set -o pipefail
mkdir -p gpurun_out/r05ab
export NT_PIPE_TRACE=1
timeout -k 10 200 python -u tools/host_pipe_probe.py --cfg3 --reps 3 > gpurun_out/r05ab/cfg3.log 2>&1 &&
unset NT_PIPE_TRACE &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "group or chunk or keyset" > gpurun_out/r05ab/tests.log 2>&1
rc=$?
grep -E "pinned|pageable|M certs" gpurun_out/r05ab/cfg3.log | head -20
tail -3 gpurun_out/r05ab/tests.log
exit $rc
