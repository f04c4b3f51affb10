#!/bin/bash
# Round 3, session 2: snapshot build traces with the caching allocator (RMAT-20 BOTH, RMAT-24 IN from ids).
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr20 -o b20 -- python3 tools/build_trace.py --scale 20 --flags 4 --reps 3 > $OUT/tr20.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr24 -o b24 -- python3 tools/build_trace.py --scale 24 --flags 2 --reps 2 > $OUT/tr24.log 2>&1 || exit 4
echo done
