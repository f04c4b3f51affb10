#!/bin/bash
# Round 3, session 2: RMAT-24 PageRank knob re-check on the current kernels (band bits, staging windows).
set -o pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 base: b0bit4:band0_bit=4 b0bit6:band0_bit=6 st64:merge_stage0=64,merge_stage1=64 st128:merge_stage0=128,merge_stage1=128 st256:merge_stage0=256,merge_stage1=256 b1deg6:band1_deg=6 b1deg12:band1_deg=12 > $OUT/ab24.json 2> $OUT/ab24.err || exit 3
timeout -k 10 500 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 2 base: st128:merge_stage0=128,merge_stage1=128 b0bit6:band0_bit=6 > $OUT/ab26.json 2> $OUT/ab26.err || exit 4
echo done
