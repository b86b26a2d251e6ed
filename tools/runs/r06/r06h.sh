#!/bin/bash
# With no short kernel waiting any more (r06g), the two pipeline streams' key-cache
# launches overlap: does one wave per SIMD per launch (NT_KEYSET_WAVES=1: twice the
# rows per wave, half the inversions) now pay on the 8-GPU shard?  Interleaved twice.
set -o pipefail
bash tools/runs/r06/ab_env.sh ${1:-r06h}/ab NT_KEYSET_WAVES 0 1 2
