set -o pipefail
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_edgestore.py tests/test_gpu_parity.py -k "edgestore or decode" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s17/pytest.log 2>&1 || exit 3
timeout -k 10 300 python tools/edgestore_bench.py --scale 20 > gpurun_out/s17/es20.json 2> gpurun_out/s17/es20.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s17/stats -o es -- python3 tools/edgestore_bench.py --scale 20 --reps 1 > gpurun_out/s17/stats.log 2>&1 || exit 5
echo done
