#!/bin/bash
# Round 3: split top-down levels (owner store + claim) — parity, A/B, per-level trace.
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "split_top_down or bfs" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/bfs_sweep.py bfs_td_split 0 2 1 0 2 > $OUT/sweep20.jsonl 2> $OUT/sweep20.err || exit 4
timeout -k 10 300 python tools/bfs_sweep.py --scale 26 bfs_td_split 0 2 0 2 > $OUT/sweep26.jsonl 2> $OUT/sweep26.err || exit 5
JG_DEBUG_BFS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/bfs20 -o bfs20 -- python3 tools/workload.py bfs20 --runs 3 > $OUT/bfs20.log 2>&1 || exit 6
echo done
