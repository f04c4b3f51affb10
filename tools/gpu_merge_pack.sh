#!/bin/bash
# Packed band entries (run on the GPU box): GPU parity suite, pr_ab variants at RMAT-24/26 (default =
# automatic width, 24-bit, 32-bit), kernel trace of the RMAT-26 A/B, then the bench line.
# Usage: bash tools/gpu_merge_pack.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/${1:-pack}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != nopytest ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
fi
SHARED=--shared-graph
V="auto: s64:merge_stage0=64 s128:merge_stage0=128 s256:merge_stage0=256 auto2:"
for S in 24 26; do
  timeout -k 10 300 python -u tools/pr_ab.py --scale $S --steps 10 --rounds 3 $SHARED $V > $OUT/ab_s$S.json 2> $OUT/ab_s$S.err || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o ab -- python3 tools/pr_ab.py --scale 26 --steps 10 --rounds 1 $SHARED $V > $OUT/stats.log 2>&1 || exit 5
#timeout -k 10 400 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 6
echo done
