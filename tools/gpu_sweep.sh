set -o pipefail
mkdir -p gpurun_out/sw26
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sw26/pytest.log 2>&1 || exit 3
timeout -k 10 400 python tools/big_configs.py --scale 22 --out gpurun_out/sw26/big22.json > gpurun_out/sw26/big22.log 2>&1 || exit 4
timeout -k 10 900 python tools/big_configs.py --scale 26 --out gpurun_out/sw26/big26.json > gpurun_out/sw26/big26.log 2>&1 || exit 5
echo done
