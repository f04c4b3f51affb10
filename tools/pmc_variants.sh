#!/bin/bash
# PMC passes (one rocprofv3 run per pass, MI355X_MICROARCH.md §rocprofv3 slot limits) over PageRank
# supersteps of bench.py for several pull-engine variants (JG_TUNE).  Usage on the GPU box:
#   bash tools/pmc_variants.sh <outdir> "<name>:<JG_TUNE>" ...
# BENCH_ARGS (env) adds bench.py arguments, e.g. BENCH_ARGS="--scale 26".
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_TAG_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_SPI_STALL_sum"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES"
  "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_RDRET_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY"
)
for v in "$@"; do
  name=${v%%:*}; tune=${v#*:}
  i=0; mkdir -p $OUT/$name
  for p in "${PASSES[@]}"; do
    JG_TUNE="$tune" timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $OUT/$name/p$i -o p -- python3 bench.py --no-cpu --no-bfs --steps 5 --warmup 1 $BENCH_ARGS > $OUT/$name/p$i.log 2>&1 || { echo "pass $i of $name failed"; exit 3; }
    i=$((i+1))
  done
done
echo done
