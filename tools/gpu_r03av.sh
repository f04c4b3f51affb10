#!/bin/bash
# Round 3, session 2: sharded CC by local union-finds + tree labels over the halo + a multi-root
# sharded DO-BFS — parity (small, multirank, RMAT-26 2/8 shards) and the 8-shard simulation.
set -o pipefail
OUT=gpurun_out/r03av
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "sharded_connected or logical_shards_match or connected_components" > $OUT/pytest.log 2>&1 || exit 2
timeout -k 10 300 python -u -m pytest tests/test_multirank_transport.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_mr.log 2>&1 || exit 3
JG_DEBUG_CC=1 timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program cc --reps 2 > $OUT/sim_cc.jsonl 2> $OUT/sim_cc.err || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cc8 -o cc8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program cc --reps 1 > $OUT/cc8.log 2>&1 || exit 5
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 500 --timeout-method thread -m gpu -k "sharded_cc" > $OUT/pytest_cfg.log 2>&1 || exit 6
echo done
