set -o pipefail
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_combine.py tests/test_gpu_computer.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s13/pytest.log 2>&1 || exit 3
timeout -k 10 200 python tools/combine_bench.py --scale 20 --steps 2 > gpurun_out/s13/comb20.json 2>&1 || exit 4
timeout -k 10 200 python tools/combine_bench.py --scale 24 --steps 10 > gpurun_out/s13/comb24.json 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s13/stats -o comb -- python3 tools/combine_bench.py --scale 24 --steps 10 > gpurun_out/s13/stats.log 2>&1 || exit 6
echo done
