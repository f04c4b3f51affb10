#!/bin/bash
# One iteration on the GPU box: a test subset, the 8-shard DO-BFS simulation traces, the bench line.
#   bash tools/gpu_iter.sh <tag> <pytest args...>
set -o pipefail
T=${1:?tag}
shift
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 13; }
tail -2 $OUT/pytest.log
timeout -k 10 600 bash tools/shard_traces.sh $OUT/st 26 8 bfs > $OUT/st.log 2>&1 || { tail -20 $OUT/st.log; exit 14; }
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 15; }
echo all-done
