#!/bin/bash
# Round 3, session 2: the 2-rank host-transport bench rehearsal on the final tree (the sharded
# union-find CC in rank mode at RMAT-26).
set -o pipefail
OUT=gpurun_out/r03ay
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 3 --warmup 1 --host-transport --no-cpu > $OUT/bench_n2.json 2> $OUT/bench_n2.err || exit 5
echo done
