#!/bin/bash
# Combiner programs on the GPU box: their GPU tests, then RMAT-24 supersteps over OUT / IN / BOTH and
# an RMAT-20 parity run.  Usage: bash tools/gpu_combine.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
OUT=gpurun_out/${1:-comb}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 3
for d in out in both; do timeout -k 10 200 python tools/combine_bench.py --scale 24 --steps 10 --direction $d >> $OUT/comb24.json 2>&1 || exit 4; done
timeout -k 10 200 python tools/combine_bench.py --scale 20 --steps 2 --direction out >> $OUT/comb20.json 2>&1 || exit 5
echo done
