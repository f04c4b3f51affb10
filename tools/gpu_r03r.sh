#!/bin/bash
# Round 3, session 2: sharded bit-parallel BFS — top-down levels, lazy forward exchange, live bits from
# the shards' own rows: parity (logical shards, rank mode, edge cases, config4), then the 8-shard
# RMAT-26 simulation (msbfs_td 1 vs 2) and its kernel trace.
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "msbfs or logical_shards or multisource" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_transport.py tests/test_gpu_edge_cases.py > $OUT/pytest2.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_configs.py -k "config4" > $OUT/pytest_configs.log 2>&1 || exit 5
timeout -k 10 300 python tools/shard_sim.py --scale 26 --shards 8 1 --program msbfs --reps 2 > $OUT/msbfs26_td1.jsonl 2> $OUT/msbfs26_td1.err || exit 6
timeout -k 10 300 python tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 2 --tune msbfs_td=2 > $OUT/msbfs26_td2.jsonl 2> $OUT/msbfs26_td2.err || exit 7
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms8 -o ms8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 1 > $OUT/ms8.log 2>&1 || exit 8
echo done
