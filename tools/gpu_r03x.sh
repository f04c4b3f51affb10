#!/bin/bash
# Round 3, session 2: hash-table id remap — builds from ids (RMAT-20/24), edgestore snapshot, GPU suite.
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 4 > $OUT/build20.json 2> $OUT/build20.err || exit 4
timeout -k 10 300 python tools/build_trace.py --scale 24 --flags 2 --reps 3 > $OUT/build24.json 2> $OUT/build24.err || exit 5
timeout -k 10 300 python tools/edgestore_bench.py --scale 20 --chunks 1,8 > $OUT/edgestore20.json 2> $OUT/edgestore20.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tr24 -o b24 -- python3 tools/build_trace.py --scale 24 --flags 2 --reps 2 > $OUT/tr24.log 2>&1 || exit 7
echo done
