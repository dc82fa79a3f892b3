#!/bin/bash
# round-end evidence in one call: the empty-batch test, part B (in-step traces, PMC) for this
# build, the traces copied into this box's profiles/ so part A's bench lines quote them, part A
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "empty_batch" > gpurun_out/r4_v.log 2>&1 || { tail -30 gpurun_out/r4_v.log; exit 1; }
tail -1 gpurun_out/r4_v.log
bash tools/gpu_final_b.sh r4b3 || exit 1
cp gpurun_out/instep_*.json profiles/ 2>/dev/null
bash tools/gpu_final_a.sh r4a3 || exit 1
