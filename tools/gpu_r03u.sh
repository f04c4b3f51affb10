#!/bin/bash
# Round 3, session 2: where a snapshot build goes (RMAT-20 from decoded ids: kernels, copies, HIP API).
set -o pipefail
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 3 > $OUT/build20.json 2> $OUT/build20.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr -o b20 -- python3 tools/build_trace.py --scale 20 --flags 4 --reps 3 > $OUT/tr.log 2>&1 || exit 4
timeout -k 10 300 python tools/edgestore_bench.py --scale 20 --chunks 1,8 > $OUT/edgestore20.json 2> $OUT/edgestore20.err || exit 5
echo done
