#!/bin/bash
# Round profile of the bench workload (run on the GPU box): bench line, rocprofv3 kernel stats of the
# same command, and PMC passes (one rocprofv3 run each, MI355X_MICROARCH.md slot limits) for the
# L2 <-> fabric traffic of every kernel of the PageRank superstep.
# Usage: bash tools/profile_round.sh <tag>   -> gpurun_out/<tag>/...
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python3 bench.py --no-cpu --no-big > $OUT/stats.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_rd -o rd -- python3 bench.py --no-cpu --no-bfs --no-big --steps 10 --warmup 2 > $OUT/pmc_rd.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wr -o wr -- python3 bench.py --no-cpu --no-bfs --no-big --steps 10 --warmup 2 > $OUT/pmc_wr.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py --no-cpu --no-bfs --no-big --steps 10 --warmup 2 > $OUT/pmc_fetch.log 2>&1 || exit 7
echo done
