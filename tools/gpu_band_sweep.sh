# PageRank pull-engine variants at RMAT-26 and RMAT-24 (tools/pr_ab.py): the empty-row skip and
# three-band splits of the heavy rows (hub band >= 2048 keeps the automatic sub-slice count).
set -o pipefail
mkdir -p gpurun_out/sw
B3="band0_deg=2048,band1_deg=128,band2_deg=8,band2_bit=3"
V="base: noskip:pr_skip_empty=0 b3s4:$B3,band1_bit=4 b3s5:$B3,band1_bit=5 b3s6:$B3,band1_bit=6 b3k1s5:band0_deg=1024,band1_deg=128,band2_deg=8,band2_bit=3,band1_bit=5"
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 3 $V > gpurun_out/sw/band_s26.json 2> gpurun_out/sw/band_s26.err || exit 3
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 $V > gpurun_out/sw/band_s24.json 2> gpurun_out/sw/band_s24.err || exit 4
echo ok
