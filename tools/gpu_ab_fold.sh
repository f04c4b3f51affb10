#!/bin/bash
# A/B of band 0 folded per (row, XCD) (Tune::ab_fold, an experiment whose ranks are not
# PageRank) against the sub-row partials, RMAT-26 and RMAT-24, interleaved in one process, plus a
# counter-free kernel trace of each variant alone.  bash tools/gpu_ab_fold.sh <out>
set -o pipefail
OUT=gpurun_out/${1:-abfold}
mkdir -p $OUT
export TMPDIR=/tmp
for sc in 26 24; do
  timeout -k 10 300 python3 tools/pr_ab.py --scale $sc --shared-graph --rounds 5 --steps 10 base:ab_fold=0 fold:ab_fold=1 > $OUT/ab$sc.json 2> $OUT/ab$sc.err || exit 3
  cat $OUT/ab$sc.json
done
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_fold$v -o t -- python3 tools/pr_ab.py --scale 26 --shared-graph --rounds 2 --steps 10 v:ab_fold=$v > $OUT/trace_fold$v.json 2> $OUT/trace_fold$v.err || exit 4
done
echo done
