#!/bin/bash
# Round 3, session 2: host index maps made on first use — GPU suite, build times (on-device RMAT, host ids), bench.
set -o pipefail
OUT=gpurun_out/r03af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/build_trace.py --scale 24 --flags 2 --reps 3 --rmat > $OUT/build24_rmat.json 2> $OUT/b1.err || exit 4
timeout -k 10 300 python tools/build_trace.py --scale 26 --flags 4 --reps 2 --rmat > $OUT/build26_rmat.json 2> $OUT/b2.err || exit 5
timeout -k 10 300 python tools/build_trace.py --scale 24 --flags 2 --reps 3 > $OUT/build24_ids.json 2> $OUT/b3.err || exit 6
timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 4 > $OUT/build20_ids.json 2> $OUT/b4.err || exit 7
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 8
echo done
