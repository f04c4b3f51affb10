set -o pipefail
mkdir -p gpurun_out/sw25
export TMPDIR=/tmp
timeout -k 10 500 python tools/pr_ab.py --rounds 7 ns_b8:pull_short=0 s_b16:pull_short=1,band1_deg=16 ns_b16:pull_short=0,band1_deg=16 s_b8:pull_short=1 s_b12:pull_short=1,band1_deg=12 > gpurun_out/sw25/ab.json 2> gpurun_out/sw25/ab.err || exit 5
echo done
