#!/bin/bash
# round 4: epilogue scale / bias loaded before the prologue (cfg 109 / 110)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "pingpong and (109 or 110)" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 8192 --cfgs 57,109,64,110 --iters 30 > $o.g8192.log 2>&1 || exit 1
cat $o.g8192.log
timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 8 "early:qkv=109,proj=110,lin1=109,lin2=110" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
