set -o pipefail
mkdir -p gpurun_out/sw11
export TMPDIR=/tmp
for d in 4096 1024 256 64 16; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw11/d$d -o st -- python3 tools/pr_ab.py --rounds 1 d$d:split_min_degree=$d > gpurun_out/sw11/d$d.log 2>&1 || exit 4
done
echo done
