#!/bin/bash
# Wave-staged DO-BFS appends (run on the GPU box): GPU parity suite, then the bench procedure's BFS
# timing with bfs_wave_stage 1 / 0 at RMAT-20, 22 and 26.  Usage: bash tools/gpu_bfs_wave.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-bfswave}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
for S in 20 22 26; do
  timeout -k 10 300 python -u tools/bfs_sweep.py --scale $S bfs_wave_stage 1 0 1 0 > $OUT/s$S.jsonl 2>&1 || exit 4
done
echo ok
