#!/bin/bash
# Round 3, session 2: DO-BFS bottom-up with two vertices per lane (bfs_bu_rows) — parity and A/B at
# RMAT-20/22/26 (bench procedure, alternating).
set -o pipefail
OUT=gpurun_out/r03az
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "bottom_up_rows or bfs_rmat or bfs_golden or split_top_down" > $OUT/pytest.log 2>&1 || exit 2
timeout -k 10 200 python tools/bfs_sweep.py bfs_bu_rows 1 2 1 2 1 2 > $OUT/ab20.jsonl 2> $OUT/ab20.err || exit 3
timeout -k 10 200 python tools/bfs_sweep.py --scale 22 bfs_bu_rows 1 2 1 2 > $OUT/ab22.jsonl 2> $OUT/ab22.err || exit 4
timeout -k 10 300 python tools/bfs_sweep.py --scale 26 bfs_bu_rows 1 2 1 2 > $OUT/ab26.jsonl 2> $OUT/ab26.err || exit 5
echo done
