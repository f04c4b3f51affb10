set -o pipefail
mkdir -p gpurun_out/sw21
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_computer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sw21/pytest.log 2>&1 || exit 3
timeout -k 10 500 python tools/pr_ab.py ovl:pull_overlap=1 noovl:pull_overlap=0 ovl6:band0_bit=6 > gpurun_out/sw21/ab.json 2> gpurun_out/sw21/ab.err || exit 5
echo done
