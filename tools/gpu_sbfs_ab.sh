#!/bin/bash
# A/B of jg_tune_set knobs on the 8-shard DO-BFS simulation traces (RMAT-26), one trace pair per setting:
#   bash tools/gpu_sbfs_ab.sh <tag> <knob=value[,knob=value]> ... ("-" = defaults; "env:VAR=value" sets an
#   environment variable for that setting instead)
# Per-shard kernel time per setting: tools/trace_diff.py over <tag>/st_<i>/bfs_{a,b} (runs from their JSON).
set -o pipefail
T=${1:?tag}
shift
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for v in "$@"; do
    args=""
    envs=""
    case "$v" in
        -) ;;
        env:*) envs="${v#env:}" ;;
        *) args="--tune ${v//,/ }" ;;
    esac
    echo "$i $v" >> $OUT/settings.txt
    env $envs SIM_ARGS="$args" timeout -k 10 600 bash tools/shard_traces.sh $OUT/st_$i 26 8 bfs > $OUT/st_$i.log 2>&1 || { tail -20 $OUT/st_$i.log; exit 14; }
    i=$((i + 1))
done
echo all-done
