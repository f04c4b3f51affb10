#!/bin/bash
# Round validation on the GPU box: the whole -m gpu suite, smoke(), the bench line and the rocprofv3
# kernel stats of the same bench command.  Usage: bash tools/gpu_final.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/${1:-f1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 4
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python3 bench.py --no-cpu > $OUT/stats.log 2>&1 || exit 6
echo done
