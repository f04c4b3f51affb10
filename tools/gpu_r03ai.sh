#!/bin/bash
# Round 3, session 2: 64-source BFS with one host read-back per level — parity; the depth-plane writes'
# cost (msbfs_diag 1: none; timing only); the one-shard kernel sequence.
set -o pipefail
OUT=gpurun_out/r03aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "msbfs or logical_shards or multisource" > $OUT/pytest.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multirank_transport.py tests/test_gpu_edge_cases.py tests/test_jni_sequence.py > $OUT/pytest2.log 2>&1 || exit 4
timeout -k 10 600 python tools/msbfs_ab.py --scale 26 --reps 3 msbfs_diag 0 0 > $OUT/diag.jsonl 2> $OUT/diag.err || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/ms1 -o ms1 -- python3 tools/workload.py msbfs26 --runs 1 > $OUT/ms1.log 2>&1 || exit 6
echo done
