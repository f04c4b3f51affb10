#!/bin/bash
# PMC traffic of the RMAT-26 PageRank superstep (the bench's headline command at --scale 26), one
# rocprofv3 run per counter pass (MI355X_MICROARCH.md slot limits).  Then:
#   python tools/pmc_summary.py gpurun_out/<tag> profiles/r02/pmc26 12
set -o pipefail
OUT=gpurun_out/${1:-pmc26}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--scale 26 --no-cpu --no-bfs --no-big --steps 10 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python3 bench.py $ARGS > $OUT/stats.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_rd -o rd -- python3 bench.py $ARGS > $OUT/pmc_rd.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wr -o wr -- python3 bench.py $ARGS > $OUT/pmc_wr.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 6
echo done
