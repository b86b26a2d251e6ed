#!/bin/bash
# One GPU session (run through gpurun) for a tree built here.  Steps, chained so
# the first failure ends the session; every GPU step under its own time limit.
#   bash tools/gpu_validate.sh <tag> [steps]      steps: any of tests smoke bench bench2 trace
# Outputs under gpurun_out/<tag>/.  Per-session variants (A/B runs, PMC
# passes) are tracked under tools/runs/<round>/, so every log a profiles/*/INDEX.md
# cites can be regenerated from the repository.
set -o pipefail
TAG=${1:?tag}
STEPS=${2:-"tests smoke bench"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
             --durations 10 > "$OUT/gpu_tests.log" 2>&1 || exit 1 ;;
    smoke) timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1 ;;
    bench) timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || exit 1 ;;
    bench2) timeout -k 10 300 python -u bench.py > "$OUT/bench2.log" 2>&1 || exit 1 ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 -u bench.py \
             > "$OUT/bench_under_rocprof.log" 2>&1 || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
