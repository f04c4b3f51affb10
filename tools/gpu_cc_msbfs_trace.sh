#!/bin/bash
# Kernel traces of CC (configs[3]) and the 64-source MS-BFS (configs[4]) at RMAT-26, one GPU.
set -o pipefail
OUT=gpurun_out/${1:-ccms}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cc -o cc -- python3 tools/cc_levels.py --scale 26 --reps 2 > $OUT/cc.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ms -o ms -- python3 tools/msbfs_levels.py --scale 26 --reps 2 > $OUT/ms.log 2>&1 || exit 4
echo ok
