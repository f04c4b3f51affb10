# Band-1 (degree 8..127) sub-slice counts and thresholds at RMAT-26, then a kernel trace with the
# light rows and the split's finalize as separate launches (fuse_finalize=0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw gpurun_out/prof
V="base: b1s4:band1_bit=4 b1s5:band1_bit=5 b1s6:band1_bit=6 b1s7:band1_bit=7 b1d16:band1_deg=16 b1d4:band1_deg=4"
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 2 $V > gpurun_out/sw/band1_s26.json 2> gpurun_out/sw/band1_s26.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/s26nf -o pr -- python3 tools/pr_ab.py --scale 26 --steps 10 --rounds 1 nofuse:fuse_finalize=0 > gpurun_out/prof/s26nf.log 2>&1 || exit 4
echo ok
