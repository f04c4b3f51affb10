#!/bin/bash
# Round 3, session 2: kernel sequence of one 64-source RMAT-26 traversal on one shard.
set -o pipefail
OUT=gpurun_out/r03ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/ms1 -o ms1 -- python3 tools/workload.py msbfs26 --runs 1 > $OUT/ms1.log 2>&1 || exit 3
echo done
