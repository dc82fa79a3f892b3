#!/bin/bash
# round 4: W4A16 ping-pong per-tile fixed cost (no-epilogue timing variants, small-K scan), the
# f16-staged transposed epilogue (cfg 104); W4A8 int8 ping-pong with spread DMA (cfg 93 vs 86)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_b
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_w8a8.py tests/test_gpu_kernels.py -m gpu -k "pingpong or w4a8_gemm" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
SAMQ_LIB=tuning timeout -k 10 300 python -u tools/bench_gemm.py --m 65536 --cfgs 57,102,104,64,103 --iters 10 > $o.noepi.log 2>&1 || exit 1
cat $o.noepi.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 8192 --cfgs 57,104 --iters 30 --shapes qkv,lin1 > $o.g8192.log 2>&1 || exit 1
cat $o.g8192.log
timeout -k 10 300 python -u tools/gemm_kscan.py 65536 57,64 64,128,256,1280 > $o.kscan.log 2>&1 || exit 1
cat $o.kscan.log
timeout -k 10 400 python -u tools/bench_cfg_ab.py 2 8 "tes:qkv=104,lin1=104" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
timeout -k 10 300 python -u tools/bench_i8.py --m 16384,65536 --cfgs 86,93 > $o.i8.log 2>&1 || exit 1
cat $o.i8.log
timeout -k 10 400 python -u tools/bench_cfg_ab_w4a8.py 2 6 > $o.ab48.log 2>&1 || exit 1
cat $o.ab48.log
