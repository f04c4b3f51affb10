set -o pipefail
mkdir -p gpurun_out/check
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/check/pytest.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/check/stats -o bench -- python bench.py --no-cpu > gpurun_out/check/stats.log 2>&1 || exit 5
echo done
