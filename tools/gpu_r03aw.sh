#!/bin/bash
# Round 3, session 2: the whole GPU suite, smoke and the bench on the tree with the sharded
# union-find CC and the 64-source BFS first-level skip; the 8-shard CC simulation.
set -o pipefail
OUT=gpurun_out/r03aw
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 3
JG_DEBUG_CC=1 timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program cc --reps 3 > $OUT/sim_cc.jsonl 2> $OUT/sim_cc.err || exit 4
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 5
echo done
