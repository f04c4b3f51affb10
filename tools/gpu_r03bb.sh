#!/bin/bash
# Round 3, session 2, final tree: whole GPU suite, smoke, bench (default command) and its rocprofv3
# kernel-trace summary.
set -o pipefail
OUT=gpurun_out/r03bb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 3
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 4
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 5
echo done
