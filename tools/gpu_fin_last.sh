# fin_last knob: parity of the variant, then A/B at RMAT-24 and RMAT-26 -> gpurun_out/fl/
set -o pipefail
mkdir -p gpurun_out/fl
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pull_engine_variants" > gpurun_out/fl/pytest.log 2>&1 || exit 3
V="base: fl:fin_last=1"
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 50 --rounds 5 $V > gpurun_out/fl/s24.json 2> gpurun_out/fl/s24.err || exit 4
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 4 $V > gpurun_out/fl/s26.json 2> gpurun_out/fl/s26.err || exit 5
echo ok
