set -o pipefail
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_jni_sequence.py::test_ctx_destroy_before_graph_is_refused tests/test_gpu_sssp_delta.py tests/test_gpu_parity.py tests/test_gpu_vdev.py tests/test_multirank_transport.py "tests/test_gpu_configs.py::test_config3_sharded_cc_and_dobfs_rmat26" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 3; }
tail -3 $OUT/pytest.log
timeout -k 10 600 bash tools/shard_traces.sh $OUT/st 26 8 bfs > $OUT/st.log 2>&1 || { tail -20 $OUT/st.log; exit 4; }
tail -5 $OUT/st.log
