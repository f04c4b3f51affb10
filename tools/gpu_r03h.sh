#!/bin/bash
# Round 3: per-level kernel durations of the single-source DO-BFS at RMAT-20 and RMAT-26.
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
JG_DEBUG_BFS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/bfs20 -o bfs20 -- python3 tools/workload.py bfs20 --runs 3 > $OUT/bfs20.log 2>&1 || exit 3
JG_DEBUG_BFS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/bfs26 -o bfs26 -- python3 tools/workload.py bfs26 --runs 2 > $OUT/bfs26.log 2>&1 || exit 4
echo done
