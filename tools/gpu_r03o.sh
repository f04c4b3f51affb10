#!/bin/bash
# Round 3, session 2: validate the tree (GPU suite, smoke, bench, kernel stats), then size what the
# merge kernels' cold gathers cost (merge_diag=4 skips them; timing only) at RMAT-24 and RMAT-26.
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 4
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python3 bench.py --no-cpu > $OUT/stats.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/diag -o ab -- python3 tools/pr_ab.py --scale 26 --steps 10 --rounds 2 base: nocold:merge_diag=4 nost:merge_diag=3 > $OUT/diag26.json 2> $OUT/diag26.err || exit 7
timeout -k 10 300 python3 tools/pr_ab.py --scale 24 --steps 10 --rounds 3 base: nocold:merge_diag=4 > $OUT/diag24.json 2> $OUT/diag24.err || exit 8
echo done
