#!/bin/bash
# Round profile: full bench line, rocprofv3 kernel stats of the same command, PMC traffic passes.
# Usage (on the GPU box): bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python bench.py --no-cpu > $OUT/stats.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python bench.py --no-cpu --no-bfs --steps 5 > $OUT/pmc_fetch.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python bench.py --no-cpu --no-bfs --steps 5 > $OUT/pmc_write.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_rdreq -o rdreq -- python bench.py --no-cpu --no-bfs --steps 5 > $OUT/pmc_rdreq.log 2>&1 || echo "rdreq pass failed (counter names)"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
echo done
