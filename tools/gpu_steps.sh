#!/bin/bash
# One GPU-box call as a list of steps, each under its own time limit; the call stops at the first step
# that fails (a fault, an abort, a time limit), so nothing else touches the GPU after it.
#
#   bash tools/gpu_steps.sh <tag> "<seconds> <name> <command ...>" ...
#
# Each step's stdout + stderr go to gpurun_out/<tag>/<name>.log.  Shorthands for <command>:
#   suite                the whole -m gpu suite (pytest -x -v, per-test timeout, thread method)
#   tests <pytest args>  a subset of it
#   smoke                __graft_entry__.smoke()
#   bench <args>         bench.py; the JSON line goes to <name>.json as well
#   trace <workload> [workload.py args]  rocprofv3 --kernel-trace --stats of tools/workload.py <workload> (no counters),
#                        summarised by tools/trace_summary.py into gpurun_out/<tag>/<name>/summary.json
#   pmc <workload>       the PMC passes of tools/pmc_workloads.sh for one workload
# Anything else runs as written (bash -c).
# Replaces the per-call tools/gpu_r0*.sh launchers of rounds 1-3.
set -o pipefail
TAG=${1:?usage: gpu_steps.sh <tag> "<seconds> <name> <command>" ...}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
    read -r secs name cmd <<< "$step"
    set -- $cmd
    kind=$1
    case "$kind" in
        suite) cmd="python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" ;;
        tests) shift; cmd="python -u -m pytest -x -v --timeout 600 --timeout-method thread $*" ;;
        smoke) cmd="python -c 'import __graft_entry__ as g; g.smoke()'" ;;
        bench) shift; cmd="python bench.py $* | tee $OUT/$name.json" ;;
        trace) shift; w=$1; shift
               cmd="rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o $w -- python3 tools/workload.py $w $* && python3 tools/trace_summary.py $OUT/$name $w" ;;
        pmc) shift; cmd="bash tools/pmc_workloads.sh $TAG/$name $1" ;;
    esac
    echo "[$(date +%T)] $name ($secs s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
    rc=$?
    tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then
        echo "step $name failed: rc=$rc"
        exit $rc
    fi
done
echo done
