#!/bin/bash
# Registry GPU tests after the lookup-ahead change, the config-3 rows with the
# registry's admission timings (NT_REG_TRACE), then the key-comb width A/B on
# this (second) box.
set -o pipefail
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_registry.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_registry.log 2>&1 || { tail -40 $OUT/gpu_registry.log; exit 1; }
tail -2 $OUT/gpu_registry.log
NT_REG_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sha --no-ingest --no-latency --no-cpu > $OUT/bench_certs.log 2> $OUT/bench_certs.err || { tail -20 $OUT/bench_certs.err; exit 1; }
grep registry $OUT/bench_certs.err
python tools/bench_brief.py $OUT/bench_certs.log
bash tools/runs/r06/ab_width.sh ${1:-r06b}/ab
