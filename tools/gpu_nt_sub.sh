# GPU suite (parity after the builder / decoder refactor), then PageRank variants: non-temporal band
# streams in the merge kernel, and band 1 with 1 / 2 / 4 sub-slices.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/gpu_suite.log 2>&1 || exit 2
V="base: nt1:merge_nt=1 nt2:merge_nt=2 nt3:merge_nt=3 b1sub1:band1_sub=1 b1sub2:band1_sub=2 b1sub4:band1_sub=4"
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 2 $V > gpurun_out/sw/ntsub_s26.json 2> gpurun_out/sw/ntsub_s26.err || exit 3
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 $V > gpurun_out/sw/ntsub_s24.json 2> gpurun_out/sw/ntsub_s24.err || exit 4
echo ok
