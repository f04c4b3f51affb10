#!/bin/bash
# Round 3: early-exit MS-BFS levels (parity + A/B), >255-level MS-BFS, RMAT-26 shard simulations.
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_edge_cases.py tests/test_gpu_neighbors.py tests/test_gpu_parity.py -k "msbfs or bfs or edge or neighbors or 255" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 380 --timeout-method thread tests/test_gpu_configs.py -k config4 > $OUT/pytest_config4.log 2>&1 || exit 4
timeout -k 10 300 python tools/msbfs_ab.py --scale 22 msbfs_bu 0 1 2 > $OUT/msbfs_ab22.jsonl 2> $OUT/msbfs_ab22.err || exit 5
timeout -k 10 400 python tools/msbfs_ab.py --scale 26 msbfs_bu 0 1 2 > $OUT/msbfs_ab26.jsonl 2> $OUT/msbfs_ab26.err || exit 6
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --halo 1 --steps 5 --warmup 1 > $OUT/pr26.jsonl 2> $OUT/pr26.err || exit 7
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 1 8 --program bfs > $OUT/bfs26.jsonl 2> $OUT/bfs26.err || exit 8
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 1 8 --program cc --reps 2 > $OUT/cc26.jsonl 2> $OUT/cc26.err || exit 9
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 1 8 --program msbfs --reps 2 > $OUT/msbfs26.jsonl 2> $OUT/msbfs26.err || exit 10
echo done
