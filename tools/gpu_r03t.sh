#!/bin/bash
# Round 3, session 2: per-kernel trace of the RMAT-20 DO-BFS workload (bench sources), with the level log.
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
JG_DEBUG_BFS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/bfs20 -o bfs20 -- python3 tools/workload.py bfs20 --runs 5 > $OUT/bfs20.log 2>&1 || exit 3
timeout -k 10 300 python tools/bfs_sweep.py bfs_batch0 10 7 8 > $OUT/batch0.jsonl 2> $OUT/batch0.err || exit 4
echo done
