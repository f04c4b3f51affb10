#!/bin/bash
# Scalar-path gather microbenchmark (tools/micro/sgather.hip), prebuilt in-tree.
set -o pipefail
mkdir -p gpurun_out/sgather
timeout -k 10 120 ./tools/micro/sgather > gpurun_out/sgather/sgather.jsonl 2>&1 || exit 3
echo done
