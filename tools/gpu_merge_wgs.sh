# merge_wgs knob: parity of the variant, then A/B at RMAT-24 and RMAT-26 -> gpurun_out/mw/
set -o pipefail
mkdir -p gpurun_out/mw
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pull_engine_variants" > gpurun_out/mw/pytest.log 2>&1 || exit 3
V="base: w2:merge_wgs=2 w2t2:merge_wgs=2,merge_temporal=2"
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 50 --rounds 5 $V > gpurun_out/mw/s24.json 2> gpurun_out/mw/s24.err || exit 4
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 4 $V > gpurun_out/mw/s26.json 2> gpurun_out/mw/s26.err || exit 5
echo ok
