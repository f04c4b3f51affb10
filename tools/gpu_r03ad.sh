#!/bin/bash
# Round 3, session 2: CC and 64-source BFS with bands cut from the column-ordered CSR vs the
# sub-slice-ordered build (same process, interleaved).
set -o pipefail
OUT=gpurun_out/r03ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/build_ab.py --scale 26 --rounds 3 col: sliced:band_sliced_build=1 > $OUT/ab26.json 2> $OUT/ab26.err || exit 3
echo done
