#!/bin/bash
# Per-workload fabric traffic (run on the GPU box): for each workload of tools/workload.py, its JSON line,
# the rocprofv3 kernel trace of the same command and one PMC pass per counter group (MI355X_MICROARCH.md
# slot limits; each pass its own run).  Then, in the build container:
#   python tools/pmc_workload_summary.py gpurun_out/<tag> profiles/<round>/pmc
# Usage: bash tools/pmc_workloads.sh <tag> [workloads...]   (default: every workload)
set -o pipefail
TAG=${1:-pmcw}
shift
WLS=${@:-bfs20 bfs26 cc26 msbfs26 pr24 pr26}
export TMPDIR=/tmp
for wl in $WLS; do
    OUT=gpurun_out/$TAG/$wl
    mkdir -p $OUT
    echo "[pmc] $wl"
    timeout -k 10 300 python3 tools/workload.py $wl > $OUT/workload.json 2> $OUT/workload.err || exit 3
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o wl -- python3 tools/workload.py $wl > $OUT/stats.log 2>&1 || exit 4
    timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/pmc_rd -o rd -- python3 tools/workload.py $wl > $OUT/pmc_rd.log 2>&1 || exit 5
    timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wr -o wr -- python3 tools/workload.py $wl > $OUT/pmc_wr.log 2>&1 || exit 6
    timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 tools/workload.py $wl > $OUT/pmc_fetch.log 2>&1 || exit 7
done
echo done
