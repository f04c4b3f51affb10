#!/bin/bash
# DO-BFS level grid (sqrt(rows) * m / 4 workgroups) with wave-staged appends, RMAT-20/22/26.
set -o pipefail
OUT=gpurun_out/${1:-bfsgridm}
mkdir -p $OUT
export TMPDIR=/tmp
for S in 20 22 26; do
  timeout -k 10 300 python -u tools/bfs_sweep.py --scale $S bfs_grid_mult 4 2 8 16 4 > $OUT/s$S.jsonl 2>&1 || exit 4
done
echo ok
