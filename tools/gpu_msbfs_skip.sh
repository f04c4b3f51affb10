#!/bin/bash
# MS-BFS merge-task skip: parity (small cases, every pull-engine variant, RMAT-26 config 4) and timing
# with the skip on / off (tools/msbfs_levels.py, RMAT-26), plus a kernel trace with it on.
set -o pipefail
OUT=gpurun_out/${1:-msskip}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread \
  -k "msbfs or multisource or variants or config4" > $OUT/pytest.log 2>&1 || exit 3
for sk in 1 0; do
  timeout -k 10 200 python3 tools/msbfs_levels.py --scale 26 --reps 3 msbfs_skip=$sk >> $OUT/ab.log 2>&1 || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms -o ms -- python3 tools/msbfs_levels.py --scale 26 --reps 2 > $OUT/ms.log 2>&1 || exit 5
echo ok
