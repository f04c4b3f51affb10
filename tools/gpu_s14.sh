set -o pipefail
mkdir -p gpurun_out/s14
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "shortest_distance or logical_shards" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s14/pytest.log 2>&1 || exit 3
echo done
