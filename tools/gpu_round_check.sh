set -o pipefail
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/stats -o bench -- python bench.py --no-cpu > gpurun_out/s3/stats.log 2>&1 || exit 5
echo done
