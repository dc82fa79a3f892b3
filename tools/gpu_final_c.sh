#!/bin/bash
# round-end evidence, part C: the grouped-weight (G = 128) and the config-4 per-GPU (B = 8, 4 lanes)
# W4A16 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --groupsize 128 > gpurun_out/r4c_bench_g128.log 2>&1 || exit 1
tail -1 gpurun_out/r4c_bench_g128.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --batch 8 > gpurun_out/r4c_bench_b8.log 2>&1 || exit 1
tail -1 gpurun_out/r4c_bench_b8.log | cut -c1-400
