#!/bin/bash
# Attention kernels: parity tests + micro-benchmark (ViT-H geometry, 2 images per launch).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 120 python tools/bench_attn.py --batch 2 --iters 20 2>&1 | grep attention
