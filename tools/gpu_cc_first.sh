#!/bin/bash
# CC (RMAT-26) union-find first-round width sweep (cc_first), with a kernel trace of each, one GPU.
set -o pipefail
OUT=gpurun_out/${1:-ccfirst}
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$k -o cc -- python3 tools/cc_levels.py --scale 26 --reps 4 cc_first=$k > $OUT/k$k.log 2>&1 || exit 3
done
echo ok
