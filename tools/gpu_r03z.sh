#!/bin/bash
# Round 3, session 2: one launch for the small per-level control buffers — GPU suite, 8-shard RMAT-26
# MS-BFS simulation and trace, bench line.
set -o pipefail
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/shard_sim.py --scale 26 --shards 8 1 --program msbfs --reps 2 > $OUT/msbfs26.jsonl 2> $OUT/msbfs26.err || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms8 -o ms8 -- python3 tools/shard_sim.py --scale 26 --shards 8 --program msbfs --reps 1 > $OUT/ms8.log 2>&1 || exit 5
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 6
echo done
