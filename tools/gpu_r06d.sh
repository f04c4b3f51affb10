set -o pipefail
T=${1:-r06d}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_vdev.py tests/test_multirank_transport.py "tests/test_gpu_configs.py::test_config3_sharded_cc_and_dobfs_rmat26" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 3; }
tail -2 $OUT/pytest.log
timeout -k 10 600 bash tools/shard_traces.sh $OUT/st 26 8 bfs > $OUT/st.log 2>&1 || { tail -20 $OUT/st.log; exit 4; }
tail -2 $OUT/st.log
timeout -k 10 900 bash tools/gpu_pmc_kernels.sh $T/pmc_ms msbfs26 --runs 3 > $OUT/pmc_ms.log 2>&1 || { tail -20 $OUT/pmc_ms.log; exit 5; }
for spec in "8 1 0" "4 2 0" "4 2 1" "2 4 0" "2 4 3"; do
  set -- $spec
  SIM_ARGS="--groups $2 --only-group $3" timeout -k 10 600 bash tools/shard_traces.sh $OUT/ms2d_p$1_g$2_$3 26 $1 msbfs > $OUT/ms2d_p$1_g$2_$3.log 2>&1 || { tail -20 $OUT/ms2d_p$1_g$2_$3.log; exit 6; }
  tail -1 $OUT/ms2d_p$1_g$2_$3.log
done
echo all-done
