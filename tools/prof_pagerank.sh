set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
JG_DEBUG_PLAN=1 timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-bfs > gpurun_out/plan.log 2>&1 || exit 3
JG_PULL_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_split -o split -- python bench.py --steps 5 --no-cpu --no-bfs > gpurun_out/prof_split.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o fetch -- python bench.py --steps 5 --no-cpu --no-bfs > gpurun_out/pmc_fetch.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o write -- python bench.py --steps 5 --no-cpu --no-bfs > gpurun_out/pmc_write.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_tcc -o tcc -- python bench.py --steps 5 --no-cpu --no-bfs > gpurun_out/pmc_tcc.log 2>&1 || exit 7
echo done
