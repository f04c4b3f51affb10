set -o pipefail
T=${1:-r06e}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_multirank_transport.py tests/test_gpu_parity.py -k "logical or sharded or multirank or ranks or bfs" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 3; }
tail -2 $OUT/pytest.log
for v in "sbfs_variant=0" "sbfs_variant=1" "sbfs_variant=2" "sbfs_variant=4" "sbfs_variant=5" "sbfs_variant=8" "dobfs_alpha=14" "dobfs_alpha=100" "dobfs_alpha=300"; do
  timeout -k 10 300 python3 tools/shard_sim.py --scale 26 --shards 8 --program bfs --reps 3 --tune $v > $OUT/sim_$v.json 2> $OUT/sim_$v.err || { tail -5 $OUT/sim_$v.err; exit 4; }
  echo "$v $(cat $OUT/sim_$v.json)"
done
echo all-done
