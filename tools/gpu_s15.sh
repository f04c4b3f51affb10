set -o pipefail
mkdir -p gpurun_out/s15
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_combine.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s15/pytest.log 2>&1 || exit 3
timeout -k 10 200 python tools/combine_bench.py --scale 24 --steps 10 > gpurun_out/s15/comb24.json 2>&1 || exit 5
echo done
