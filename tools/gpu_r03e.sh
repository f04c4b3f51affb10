#!/bin/bash
# Round 3: adaptive BFS batch A/B, byte depth planes (parity + timing), RMAT-26 shard simulation.
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py -k "config4 or config1" tests/test_gpu_parity.py -k "msbfs or bfs or config" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/bfs_sweep.py bfs_adaptive_batch 0 1 0 1 > $OUT/bfs20_adaptive.jsonl 2> $OUT/bfs20_adaptive.err || exit 4
timeout -k 10 300 python tools/bfs_sweep.py --scale 26 bfs_adaptive_batch 0 1 > $OUT/bfs26_adaptive.jsonl 2> $OUT/bfs26_adaptive.err || exit 5
timeout -k 10 300 python tools/workload.py msbfs26 --runs 3 > $OUT/msbfs26.json 2> $OUT/msbfs26.err || exit 6
timeout -k 10 600 python tools/shard_sim.py --scale 26 --shards 1 8 --steps 5 --warmup 1 > $OUT/shard_sim26.jsonl 2> $OUT/shard_sim26.err || exit 7
echo done
