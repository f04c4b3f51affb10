#!/bin/bash
# CC (RMAT-26): direction-rule sweep of the multi-root eccentricity BFS (bfs_alpha / bfs_beta), one GPU.
set -o pipefail
OUT=gpurun_out/${1:-ccalpha}
mkdir -p $OUT
for kv in bfs_alpha=14 bfs_alpha=8 bfs_alpha=20 bfs_alpha=30 bfs_alpha=50 bfs_beta=12 bfs_beta=48; do
  timeout -k 10 200 python3 tools/cc_levels.py --scale 26 --reps 4 $kv >> $OUT/sweep.log 2>&1 || exit 3
done
echo ok
