#!/bin/bash
set -o pipefail
OUT=gpurun_out/split
mkdir -p $OUT
export TMPDIR=/tmp
JG_DEBUG_SPLIT=1 timeout -k 10 200 python tools/pr_variants.py --rounds 1 --variants 4:0:1,4:0:2 > $OUT/dbg.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python tools/pr_variants.py --rounds 2 --variants 4:0:0,4:0:1,4:0:2 > $OUT/trace.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o t -- python tools/pr_variants.py --rounds 1 --variants 4:0:0,4:0:1,4:0:2 > $OUT/tcc.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o t -- python tools/pr_variants.py --rounds 1 --variants 4:0:0,4:0:1,4:0:2 > $OUT/fetch.log 2>&1 || exit 6
echo done
