# rocprofv3 kernel trace of PageRank supersteps at RMAT-24 and RMAT-26 (tools/pr_ab.py, default knobs,
# or the variant given as $1): per-kernel durations of the superstep's launch sequence.
set -o pipefail
export TMPDIR=/tmp
V=${1:-base:}
mkdir -p gpurun_out/prof
for S in 26 24; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/s$S -o pr -- python3 tools/pr_ab.py --scale $S --steps 10 --rounds 1 $V > gpurun_out/prof/s$S.log 2>&1 || exit 3
done
echo ok
