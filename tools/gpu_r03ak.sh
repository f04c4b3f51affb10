#!/bin/bash
# Round 3, session 2: 64-source BFS — task bitmaps skipped on the first pull level (A/B), and the
# 8-shard RMAT-26 simulation with the per-level depth words.
set -o pipefail
OUT=gpurun_out/r03ak
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/msbfs_ab.py --scale 26 --reps 3 msbfs_skip_first 0 1 0 1 > $OUT/skip_first.jsonl 2> $OUT/skip_first.err || exit 3
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 2 > $OUT/sim_msbfs.jsonl 2> $OUT/sim_msbfs.err || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms8 -o ms8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 1 > $OUT/ms8.log 2>&1 || exit 5
echo done
