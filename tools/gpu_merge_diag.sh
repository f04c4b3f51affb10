#!/bin/bash
# Merge-kernel diagnostics + light-row degree runs (run on the GPU box): GPU parity suite, then
# pr_ab variants at RMAT-24 and RMAT-26.  Usage: bash tools/gpu_merge_diag.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
for S in 24 26; do
  timeout -k 10 300 python -u tools/pr_ab.py --scale $S --steps 10 --rounds 3 base: noruns:light_runs=0 stage:merge_diag=1 dup:merge_diag=2 nost:merge_diag=3 > $OUT/ab_s$S.json 2> $OUT/ab_s$S.err || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o ab -- python3 tools/pr_ab.py --scale 26 --steps 10 --rounds 1 base: noruns:light_runs=0 stage:merge_diag=1 dup:merge_diag=2 nost:merge_diag=3 > $OUT/stats.log 2>&1 || exit 5
echo done
