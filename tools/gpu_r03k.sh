#!/bin/bash
# Round 3: per-level trace of the bench's 6 RMAT-20 sources; split bounds at RMAT-26.
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
S0="bfs_td_split=0"
S2="bfs_td_split=2,bfs_td_split_levels=2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t20 -o t20 -- python3 tools/bfs_ab.py --scale 20 --rounds 1 $S0 > $OUT/t20.log 2>&1 || exit 3
timeout -k 10 400 python tools/bfs_ab.py --scale 26 --rounds 2 $S0 $S2 > $OUT/ab26.jsonl 2> $OUT/ab26.err || exit 4
timeout -k 10 300 python tools/bfs_ab.py --scale 20 --rounds 5 $S0 $S2 > $OUT/ab20.jsonl 2> $OUT/ab20.err || exit 5
echo done
