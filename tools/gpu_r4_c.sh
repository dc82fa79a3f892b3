#!/bin/bash
# round 4: in-graph upper bound of the GEMM epilogues (timing-only no-epilogue cfgs 102 / 103 of the
# tuning build in the 2-lane W4A16 graph; outputs wrong on purpose)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_c
SAMQ_LIB=tuning timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 6 "noepi:qkv=102,proj=103,lin1=102,lin2=103;noepi_res:proj=103,lin2=103;noepi_f16:qkv=102,lin1=102" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_w4a8.py -m gpu -k "rel_attention_q_out or stage_local" > $o.w4a8.log 2>&1 || { tail -60 $o.w4a8.log; exit 1; }
grep -E "off by one|passed|failed" $o.w4a8.log
