#!/bin/bash
# Round validation on the GPU box: the -m gpu suite, smoke(), the bench line, the bench process under a
# counter-free kernel trace cut to its timed windows (tools/bench_trace.py), the 8-shard DO-BFS
# simulation traces and the PMC passes of the bench's workloads (tools/pmc_workloads.sh).
#   bash tools/gpu_final.sh <tag> [head sha]   ->  gpurun_out/<tag>/
set -o pipefail
T=${1:?tag}
export JG_BENCH_HEAD=${2:-}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/suite.log 2>&1 || { tail -30 $OUT/suite.log; exit 13; }
tail -2 $OUT/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 14; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 15; }
JG_TRACE_MARKS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o bench -- python3 bench.py --no-cpu --trace-windows > $OUT/bench_traced.json 2> $OUT/bench_traced.err || { tail -20 $OUT/bench_traced.err; exit 16; }
timeout -k 10 600 bash tools/shard_traces.sh $OUT/st 26 8 bfs > $OUT/st.log 2>&1 || { tail -20 $OUT/st.log; exit 17; }
[ -n "$PMC" ] && { timeout -k 10 1500 bash tools/pmc_workloads.sh $T/pmc $PMC > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 18; }; }
echo all-done
