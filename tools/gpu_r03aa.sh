#!/bin/bash
# Round 3, session 2: exchange timing of every sharded program (ExchTimer) — parity, 8-shard RMAT-26
# simulations with exchange_ms, and the 2-rank host-transport bench rehearsal's per_rank blocks.
set -o pipefail
OUT=gpurun_out/r03aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_multirank_transport.py > $OUT/pytest.log 2>&1 || exit 3
for P in msbfs cc bfs pr; do
  timeout -k 10 400 python tools/shard_sim.py --scale 26 --shards 8 --program $P --reps 2 --halo 1 > $OUT/sim_$P.jsonl 2> $OUT/sim_$P.err || exit 4
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 3 --warmup 1 --host-transport --no-cpu > $OUT/bench_n2.json 2> $OUT/bench_n2.err || exit 5
echo done
