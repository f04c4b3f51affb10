#!/bin/bash
# DO-BFS tail fixes (run on the GPU box): GPU parity suite, then the bench procedure's BFS timing with
# each of bfs_init_suffix / bfs_grow_rule / bfs_batch0 switched back, at RMAT-20, 22 and 26.
set -o pipefail
OUT=gpurun_out/${1:-bfstail}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
for S in 20 22 26; do
  timeout -k 10 300 python -u tools/bfs_sweep.py --scale $S bfs_init_suffix 1 0 1 0 > $OUT/init_s$S.jsonl 2>&1 || exit 4
  timeout -k 10 300 python -u tools/bfs_sweep.py --scale $S bfs_grow_rule 1 0 1 0 > $OUT/grow_s$S.jsonl 2>&1 || exit 5
  timeout -k 10 300 python -u tools/bfs_sweep.py --scale $S bfs_batch0 10 8 10 8 > $OUT/batch_s$S.jsonl 2>&1 || exit 6
done
echo ok
