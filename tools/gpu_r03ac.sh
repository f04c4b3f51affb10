#!/bin/bash
# Round 3, session 2: bands cut from the column-ordered CSR (one select + sort instead of two) —
# GPU suite, build times, PageRank A/B against the sub-slice-ordered build, bench line.
set -o pipefail
OUT=gpurun_out/r03ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/build_trace.py --scale 20 --flags 4 --reps 4 > $OUT/build20.json 2> $OUT/build20.err || exit 4
timeout -k 10 300 python tools/build_trace.py --scale 24 --flags 2 --reps 3 > $OUT/build24.json 2> $OUT/build24.err || exit 5
timeout -k 10 500 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 colbuild: sliced:band_sliced_build=1 > $OUT/ab24.json 2> $OUT/ab24.err || exit 6
timeout -k 10 500 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 2 colbuild: sliced:band_sliced_build=1 > $OUT/ab26.json 2> $OUT/ab26.err || exit 7
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 8
echo done
