#!/bin/bash
# Round 3, session 2: sparse reverse exchange of the sharded bit-parallel BFS — parity, 8-shard RMAT-26
# simulation (sparse vs dense reverse) with the level log, and its kernel trace.
set -o pipefail
OUT=gpurun_out/r03ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "msbfs or logical_shards or multisource" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_transport.py tests/test_gpu_edge_cases.py > $OUT/pytest2.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_configs.py -k "config4" > $OUT/pytest_configs.log 2>&1 || exit 5
timeout -k 10 300 python tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 2 > $OUT/msbfs26_sparse.jsonl 2> $OUT/msbfs26_sparse.err || exit 6
timeout -k 10 300 python tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 2 --tune msbfs_sparse=0 > $OUT/msbfs26_dense.jsonl 2> $OUT/msbfs26_dense.err || exit 7
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms8 -o ms8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 1 > $OUT/ms8.log 2>&1 || exit 8
echo done
