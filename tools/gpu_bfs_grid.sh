#!/bin/bash
# Per-level kernel traces of single-source DO-BFS at RMAT-20 for several level grids (run on the GPU
# box; tools/bfs_levels.py + rocprofv3 kernel trace).  Usage: bash tools/gpu_bfs_grid.sh -> gpurun_out/bfsgrid/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/bfsgrid
mkdir -p $OUT
for G in 128 256 1024 4096; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/g$G -o bfs -- python3 tools/bfs_levels.py --scale 20 --runs 4 --tune bfs_grid=$G > $OUT/g$G.log 2>&1 || exit 3
done
echo ok
