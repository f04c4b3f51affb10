#!/bin/bash
# Round 3: sharded DO-BFS with bit-packed frontier exchange — parity, shard simulation; RMAT-20 level trace.
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "logical_shards or bfs" tests/test_multirank_transport.py tests/test_gpu_edge_cases.py > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_configs.py -k "sharded" > $OUT/pytest_configs.log 2>&1 || exit 4
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program bfs --reps 2 > $OUT/bfs26_p8.jsonl 2> $OUT/bfs26_p8.err || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bfs8 -o bfs8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program bfs --reps 1 > $OUT/bfs8.log 2>&1 || exit 6
S0="bfs_td_split=0"
S2="bfs_td_split=2,bfs_td_split_levels=2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t20 -o t20 -- python3 tools/bfs_ab.py --scale 20 --rounds 1 $S0 > $OUT/t20.log 2>&1 || exit 7
timeout -k 10 400 python tools/bfs_ab.py --scale 26 --rounds 2 $S0 $S2 > $OUT/ab26.jsonl 2> $OUT/ab26.err || exit 8
echo done
