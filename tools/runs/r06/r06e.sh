#!/bin/bash
# After the key-set width fallback: the key-cache tests and the full-size
# two-rank rehearsal on one GPU (two processes sharing its HBM).
set -o pipefail
OUT=gpurun_out/${1:-r06e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_memory.py tests/test_wire.py -x -q --timeout 300 --timeout-method thread -m gpu -k "keyset or budget or ingest or core" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
NT_BENCH_DEVICE=0 timeout -k 10 500 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > $OUT/bench_2ranks.log 2> $OUT/bench_2ranks.err || { grep -n "Error\|error" $OUT/bench_2ranks.err | head -20; exit 1; }
python tools/bench_brief.py $OUT/bench_2ranks.log > $OUT/brief.txt; cat $OUT/brief.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2> $OUT/bench20.err || { tail -20 $OUT/bench20.err; exit 1; }
python tools/bench_brief.py $OUT/bench20.log
