#!/bin/bash
# MS-BFS (RMAT-26, BOTH plan): hub-band sub-slice bits sweep (0 = automatic), one GPU.
set -o pipefail
OUT=gpurun_out/${1:-msbits}
mkdir -p $OUT
for b in 0 6 7 8; do
  timeout -k 10 200 python3 tools/msbfs_levels.py --scale 26 --reps 3 band0_bit=$b >> $OUT/sweep.log 2>&1 || exit 3
done
for b in 3 4 5; do
  timeout -k 10 200 python3 tools/msbfs_levels.py --scale 26 --reps 3 band1_bit=$b >> $OUT/sweep.log 2>&1 || exit 4
done
echo ok
