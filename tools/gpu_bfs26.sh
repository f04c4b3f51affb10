# Per-level DO-BFS at RMAT-26: kernel trace (durations) and the level log (direction, frontier).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bfs26
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bfs26/trace -o bfs -- python3 tools/bfs_levels.py --scale 26 --runs 3 > gpurun_out/bfs26/trace.log 2>&1 || exit 3
JG_DEBUG_BFS=1 timeout -k 10 200 python3 tools/bfs_levels.py --scale 26 --runs 3 > gpurun_out/bfs26/levels.log 2>&1 || exit 4
echo ok
