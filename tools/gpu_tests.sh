#!/bin/bash
# Run a subset of the -m gpu suite on the GPU box: bash tools/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
OUT=gpurun_out/${1:-t}
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
exit $rc
