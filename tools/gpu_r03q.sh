#!/bin/bash
# Round 3, session 2: rank-mode transport tests, and the kernel trace of the 8-shard RMAT-26 MS-BFS simulation.
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_transport.py tests/test_gpu_edge_cases.py > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/ms8 -o ms8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 1 > $OUT/ms8.log 2>&1 || exit 4
echo done
