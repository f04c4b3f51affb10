#!/bin/bash
# bench.py's N > 1 path rehearsed on one GPU: N ranks under torch.distributed.run, every rank on
# device 0, exchanges over gloo through the library's host transport (not a measurement).
#   bash tools/gpu_bench_rehearsal.sh <out name> <git head of the uploaded tree>
# N = 2 runs the default CC plan (replicated: every rank builds the whole graph), N = 8 the sharded one
# (--cc-plan sharded): eight whole RMAT-26 builds do not fit one GPU, they need one GPU per rank.
set -o pipefail
OUT=gpurun_out/${1:-rehearsal}
mkdir -p $OUT
echo "${2:-unknown}" > $OUT/head
export TMPDIR=/tmp
for N in 2 8; do
  extra=""
  [ $N = 8 ] && extra="--cc-plan sharded"
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --host-transport --no-cpu $extra > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err || exit 3
done
echo ok
