#!/bin/bash
# MS-BFS (configs[4], RMAT-26): top-down/pull switch threshold sweep (bfs_alpha), one GPU.
set -o pipefail
OUT=gpurun_out/${1:-msalpha}
mkdir -p $OUT
for a in 14 7 4 2 1; do
  timeout -k 10 200 python3 tools/msbfs_levels.py --scale 26 --reps 2 bfs_alpha=$a >> $OUT/sweep.log 2>&1 || exit 3
done
echo ok
