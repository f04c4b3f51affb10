# Iteration check: GPU parity suite, BFS trace at RMAT-20, PageRank rank-store variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/gpu_suite.log 2>&1 || exit 2
bash tools/gpu_bfs_trace.sh || exit 3
V="base: rankall:pr_rank_last=0"
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 3 $V > gpurun_out/sw/rank_s26.json 2> gpurun_out/sw/rank_s26.err || exit 4
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 $V > gpurun_out/sw/rank_s24.json 2> gpurun_out/sw/rank_s24.err || exit 5
timeout -k 10 300 python -u bench.py --no-cpu --no-big --steps 20 > gpurun_out/sw/bench_quick.json 2> gpurun_out/sw/bench_quick.err || exit 6
echo ok
