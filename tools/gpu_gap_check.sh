# superstep gaps without the per-superstep profiling events: kernel trace of tools/pr_ab.py -> gpurun_out/gap/
set -o pipefail
mkdir -p gpurun_out/gap
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/t -o pr -- python3 tools/pr_ab.py --scale 24 --steps 20 --rounds 2 base: > gpurun_out/gap/log 2>&1 || exit 3
echo ok
