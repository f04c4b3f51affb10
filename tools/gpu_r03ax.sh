#!/bin/bash
# Round 3, session 2: sharded CC fallback (no bounded search) parity, and the msbfs suite after the
# unused-counter cleanup.
set -o pipefail
OUT=gpurun_out/r03ax
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread -m gpu -k "sharded_connected or msbfs or logical_shards_match" > $OUT/pytest.log 2>&1 || exit 2
echo done
