# Kernel trace of single-source DO-BFS at RMAT-20 (per-level kernel durations and the gaps between
# them; tools/bfs_levels.py), then the levels of each run (JG_DEBUG_BFS=1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bfs
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bfs/trace -o bfs -- python3 tools/bfs_levels.py --scale 20 --runs 4 > gpurun_out/bfs/trace.log 2>&1 || exit 3
JG_DEBUG_BFS=1 timeout -k 10 100 python3 tools/bfs_levels.py --scale 20 --runs 2 > gpurun_out/bfs/levels.log 2>&1 || exit 4
echo ok
