set -o pipefail
mkdir -p gpurun_out/sw14
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_computer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sw14/pytest.log 2>&1 || exit 3
timeout -k 10 400 python tools/pr_ab.py plain:pull_split=0 nolds:slice_lds=0 d64:split_min_degree=64 d32:split_min_degree=32 d16:split_min_degree=16 d8:split_min_degree=8 > gpurun_out/sw14/ab.json 2> gpurun_out/sw14/ab.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw14/st -o st -- python3 tools/pr_slice_locality.py --ks 14 > gpurun_out/sw14/st.log 2>&1 || exit 4
echo done
