#!/bin/bash
# Round 3: split top-down level policy A/B on the bench's sources (RMAT-20, 26), level logs.
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
S0="bfs_td_split=0"
S1="bfs_td_split=2,bfs_td_split_levels=2,bfs_td_split_min=65536"
S2="bfs_td_split=2,bfs_td_split_levels=6,bfs_td_split_min=65536"
S3="bfs_td_split=2,bfs_td_split_levels=7,bfs_td_split_min=65536"
S4="bfs_td_split=2,bfs_td_split_levels=6,bfs_td_split_min=16384"
timeout -k 10 300 python tools/bfs_ab.py --scale 20 --rounds 5 $S0 $S1 $S2 $S3 $S4 > $OUT/ab20.jsonl 2> $OUT/ab20.err || exit 3
JG_DEBUG_BFS=1 timeout -k 10 300 python tools/bfs_ab.py --scale 20 --rounds 1 $S0 > $OUT/levels20.jsonl 2> $OUT/levels20.err || exit 4
timeout -k 10 400 python tools/bfs_ab.py --scale 26 --rounds 2 $S0 $S2 > $OUT/ab26.jsonl 2> $OUT/ab26.err || exit 5
echo done
