#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "empty_batch" > gpurun_out/r4_v.log 2>&1; rc=$?; tail -30 gpurun_out/r4_v.log; exit $rc
