#!/bin/bash
# Round 3, session 2: caching device allocator — snapshot build times (cache on / off), the GPU suite.
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 4 > $OUT/build20.json 2> $OUT/build20.err || exit 3
JG_NO_DEVCACHE=1 timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 4 > $OUT/build20_nocache.json 2> $OUT/build20_nocache.err || exit 4
timeout -k 10 300 python tools/build_trace.py --scale 24 --flags 2 --reps 3 > $OUT/build24.json 2> $OUT/build24.err || exit 5
timeout -k 10 300 python tools/edgestore_bench.py --scale 20 --chunks 1,8 > $OUT/edgestore20.json 2> $OUT/edgestore20.err || exit 6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 7
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 8
echo done
