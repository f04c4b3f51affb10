#!/bin/bash
# Round 3, session 2: msbfs_skip_first on by default — 64-source BFS parity and the sharded simulation.
set -o pipefail
OUT=gpurun_out/r03al
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread -m gpu -k "msbfs or abi" > $OUT/pytest.log 2>&1 || exit 2
timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 2 > $OUT/sim_msbfs.jsonl 2> $OUT/sim_msbfs.err || exit 4
timeout -k 10 500 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 5
echo done
