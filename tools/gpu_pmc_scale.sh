#!/bin/bash
# Fabric traffic per kernel of the RMAT-$SCALE (default 26) PageRank superstep (tools/pr_ab.py, default knobs): one
# rocprofv3 PMC pass each for the read-request size split and the write requests (MI355X_MICROARCH.md
# slot limits), summarised per kernel and launch slot by tools/pmc_table.py.
# Usage on the GPU box: [SCALE=24] bash tools/gpu_pmc_scale.sh [variant spec for pr_ab.py]
set -o pipefail
export TMPDIR=/tmp
V=${1:-base:}
S=${SCALE:-26}
OUT=gpurun_out/pmc$S/${V%%:*}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/p0 -o p -- python3 tools/pr_ab.py --scale $S --steps 4 --rounds 1 $V > $OUT/p0.log 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/p1 -o p -- python3 tools/pr_ab.py --scale $S --steps 4 --rounds 1 $V > $OUT/p1.log 2>&1 || exit 4
python3 tools/pmc_table.py gpurun_out/pmc$S --per-step pull_merge_kernel=2 PrOp > gpurun_out/pmc$S/table.json || exit 5
echo ok
