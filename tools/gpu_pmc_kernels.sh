#!/bin/bash
# Per-kernel PMC of one tools/workload.py workload (the 64-source BFS's merge kernel):
# L2 hit/miss, fabric read requests by size and write requests, each group in its own pass
# (MI355X_MICROARCH.md slot limits), plus a counter-free kernel trace of the same command.
#   bash tools/gpu_pmc_kernels.sh <tag> <workload> [--runs R]   ->  gpurun_out/<tag>/
# Summarise in the build container: python tools/pmc_kernel_summary.py gpurun_out/<tag>
set -o pipefail
TAG=${1:?tag}
WL=${2:?workload}
shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 tools/workload.py $WL "$@" > $OUT/trace.json 2> $OUT/trace.err || exit 3
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_hit -o p -- python3 tools/workload.py $WL "$@" > $OUT/pmc_hit.json 2> $OUT/pmc_hit.err || exit 4
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_rd -o p -- python3 tools/workload.py $WL "$@" > $OUT/pmc_rd.json 2> $OUT/pmc_rd.err || exit 5
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wr -o p -- python3 tools/workload.py $WL "$@" > $OUT/pmc_wr.json 2> $OUT/pmc_wr.err || exit 6
echo done
