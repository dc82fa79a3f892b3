#!/bin/bash
# round 4: persistent ping-pong GEMMs (cfg 107 / 108): stores drain under the next tile's prologue
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_f
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "pingpong or persistent" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 8192 --cfgs 57,107,64,108 --iters 30 > $o.g8192.log 2>&1 || exit 1
cat $o.g8192.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 65536 --cfgs 57,107,64,108 --iters 10 > $o.g65536.log 2>&1 || exit 1
cat $o.g65536.log
timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 8 "persist:qkv=107,proj=108,lin1=107,lin2=108;persist_f16:qkv=107,lin1=107;persist_res:proj=108,lin2=108" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
