#!/bin/bash
# Round 3, session 2: kernel trace of the on-device RMAT builds (RMAT-24 IN, RMAT-26 BOTH), second build of each.
set -o pipefail
OUT=gpurun_out/r03ae
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/t24 -o b24 -- python3 tools/build_trace.py --scale 24 --flags 2 --reps 2 --rmat > $OUT/t24.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/t26 -o b26 -- python3 tools/build_trace.py --scale 26 --flags 4 --reps 2 --rmat > $OUT/t26.log 2>&1 || exit 4
echo done
