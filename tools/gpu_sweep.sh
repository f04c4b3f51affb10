set -o pipefail
mkdir -p gpurun_out/sw19
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sw19/pytest.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > gpurun_out/sw19/bench.json 2> gpurun_out/sw19/bench.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw19/stats -o bench -- python bench.py --no-cpu > gpurun_out/sw19/stats.log 2>&1 || exit 5
echo done
