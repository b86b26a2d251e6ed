set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ac
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05ac/tr -o run -- python3 -u tools/host_pipe_probe.py --cfg3 --reps 3 > gpurun_out/r05ac/probe.log 2>&1
rc=$?
find gpurun_out/r05ac -name "*.csv" | head
exit $rc
