#!/bin/bash
# Per-shard kernel time of the P-logical-shard simulation (tools/shard_sim.py) from counter-free kernel
# traces: each program is traced twice with different repetition counts, and tools/trace_diff.py (run in
# the build container) takes the difference, so build kernels and warm-up calls cancel out.
#   bash tools/shard_traces.sh <out dir> <scale> <shards> [programs...]   (default: pr bfs cc msbfs)
# -> <out dir>/<program>_{a,b}/ (traces) and <program>_{a,b}.json (shard_sim's line: its "runs")
# SIM_ARGS (environment): extra shard_sim.py arguments, e.g. "--groups 2 --only-group 1" (a 2D plan's group)
set -o pipefail
OUT=${1:?out dir}
SCALE=${2:-26}
P=${3:-8}
shift 3
PROGS=${@:-pr bfs cc msbfs}
export TMPDIR=/tmp
mkdir -p "$OUT"
for prog in $PROGS; do
    for v in a b; do
        if [ "$prog" = pr ]; then
            steps=$([ $v = a ] && echo 4 || echo 12)
            args="--program pr --steps $steps --warmup 2 --halo 1"
        else
            reps=$([ $v = a ] && echo 1 || echo 3)
            args="--program $prog --reps $reps"
        fi
        echo "[shard_traces] $prog $v: $args"
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${prog}_$v" -o t -- \
            python3 tools/shard_sim.py --scale "$SCALE" --shards "$P" $args $SIM_ARGS > "$OUT/${prog}_$v.json" 2> "$OUT/${prog}_$v.err" || exit 3
        tail -n 1 "$OUT/${prog}_$v.json"
    done
done
echo done
