set -euo pipefail
OUT=gpurun_out/pmc_ks
mkdir -p $OUT
export TMPDIR=/tmp
PMC_BENCH_ARGS="--no-sha --no-ingest --sigs 65536" bash tools/pmc_collect.sh $OUT
