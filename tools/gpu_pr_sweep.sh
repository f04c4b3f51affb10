set -o pipefail
mkdir -p gpurun_out/sw
V="base: u8:pull_unroll=8 nt:pull_nt=1 t0:merge_temporal=0 t2:merge_temporal=2 b0bit5:band0_bit=5 b0bit6:band0_bit=6 b1bit4:band1_bit=4"
timeout -k 10 400 python -u tools/pr_ab.py --scale 26 --steps 10 --rounds 3 $V > gpurun_out/sw/s26.json 2> gpurun_out/sw/s26.err || exit 3
timeout -k 10 300 python -u tools/pr_ab.py --scale 24 --steps 20 --rounds 3 $V > gpurun_out/sw/s24.json 2> gpurun_out/sw/s24.err || exit 4
echo ok
