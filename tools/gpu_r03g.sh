#!/bin/bash
# Round 3: MS-BFS early-exit threshold sweep; kernel trace of the 8-shard DO-BFS / MS-BFS / CC at RMAT-26.
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/msbfs_ab.py --scale 22 msbfs_bu_frac 200 300 400 500 700 900 > $OUT/frac22.jsonl 2> $OUT/frac22.err || exit 3
timeout -k 10 500 python tools/msbfs_ab.py --scale 26 --reps 2 msbfs_bu_frac 300 400 500 700 > $OUT/frac26.jsonl 2> $OUT/frac26.err || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bfs8 -o bfs8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program bfs --reps 1 > $OUT/bfs8.log 2>&1 || exit 5
echo done
