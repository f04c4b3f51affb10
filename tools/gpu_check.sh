#!/bin/bash
# A whole-round check on the GPU box: the -m gpu suite, smoke(), the 8-shard DO-BFS simulation traces, the
# bench line, and the bench process under a counter-free kernel trace with its timed windows
# (tools/bench_trace.py).   bash tools/gpu_check.sh <tag> [head sha]
set -o pipefail
T=${1:?tag}
export JG_BENCH_HEAD=${2:-}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/suite.log 2>&1 || { tail -30 $OUT/suite.log; exit 3; }
tail -2 $OUT/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 4; }
timeout -k 10 600 bash tools/shard_traces.sh $OUT/st 26 8 bfs > $OUT/st.log 2>&1 || { tail -20 $OUT/st.log; exit 5; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 6; }
JG_TRACE_MARKS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o bench -- python3 bench.py --no-cpu --trace-windows > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { tail -20 $OUT/bench_traced.err; exit 7; }
echo all-done
