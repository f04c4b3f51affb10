#!/bin/bash
# LDS-staged partial stores of the merge kernel (run on the GPU box): GPU parity suite, then pr_ab
# variants at RMAT-24 and RMAT-26, and the kernel trace of the RMAT-26 A/B.
# Usage: bash tools/gpu_merge_stage.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/${1:-stage}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
V="auto: off:merge_stage0=0,merge_stage1=0 st256:merge_stage0=256,merge_stage1=256 st64:merge_stage0=64,merge_stage1=64 reload:merge_diag=2 noruns:light_runs=0"
for S in 24 26; do
  timeout -k 10 300 python -u tools/pr_ab.py --scale $S --steps 10 --rounds 3 $V > $OUT/ab_s$S.json 2> $OUT/ab_s$S.err || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o ab -- python3 tools/pr_ab.py --scale 26 --steps 10 --rounds 1 $V > $OUT/stats.log 2>&1 || exit 5
echo done
