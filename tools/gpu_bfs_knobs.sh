# DO-BFS knob sweeps at RMAT-20 (grid, Beamer alpha / beta) and the sharded PageRank simulation at
# RMAT-24, P = 8 (per-shard compute and exchange time on one GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/knobs
timeout -k 10 200 python -u tools/bfs_sweep.py bfs_grid 256 512 1024 2048 4096 > gpurun_out/knobs/grid.jsonl 2>&1 || exit 3
timeout -k 10 200 python -u tools/bfs_sweep.py bfs_alpha 6 10 14 20 30 > gpurun_out/knobs/alpha.jsonl 2>&1 || exit 4
timeout -k 10 200 python -u tools/bfs_sweep.py bfs_beta 12 24 48 96 > gpurun_out/knobs/beta.jsonl 2>&1 || exit 5
timeout -k 10 300 python -u tools/shard_sim.py --scale 24 --shards 8 --steps 10 > gpurun_out/knobs/shard_sim.json 2> gpurun_out/knobs/shard_sim.err || exit 6
echo ok
