#!/bin/bash
# round 4: residual adds moved from the GEMM epilogues into the LayerNorms (engine.res_mode)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_d
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_encoder.py -m gpu -k "add_layernorm or residual_add" > $o.tests.log 2>&1 || { tail -60 $o.tests.log; exit 1; }
grep -E "parity|passed|failed" $o.tests.log
timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 8 "ln32:res=ln32;ln16:res=ln16" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
timeout -k 10 400 python -u tools/bench_cfg_ab_w4a8.py 2 6 > $o.ab48.log 2>&1 || exit 1
cat $o.ab48.log
