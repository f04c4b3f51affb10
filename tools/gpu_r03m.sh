#!/bin/bash
# Round 3: sharded DO-BFS with bit-packed frontiers (stamped marks, wave-staged appends) — parity, simulation.
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "logical_shards or bfs" tests/test_multirank_transport.py tests/test_gpu_edge_cases.py > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_configs.py -k "sharded" > $OUT/pytest_configs.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bfs8 -o bfs8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program bfs --reps 2 > $OUT/bfs8.log 2>&1 || exit 5
echo done
