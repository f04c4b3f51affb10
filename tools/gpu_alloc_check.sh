#!/bin/bash
# Scratch allocated before the timed regions: BFS/CC/MS-BFS parity and the first-call vs later-call times.
set -o pipefail
OUT=gpurun_out/${1:-alloc}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread \
  -k "msbfs or multisource or bfs or cc or connected or config" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 200 python3 tools/cc_levels.py --scale 26 --reps 3 >> $OUT/t.log 2>&1 || exit 4
timeout -k 10 200 python3 tools/msbfs_levels.py --scale 26 --reps 3 >> $OUT/t.log 2>&1 || exit 5
echo ok
