#!/bin/bash
# round 4: LDS-DMA pieces spread through the MFMA burst (cfg 100 / 101 vs 57 / 64); grouped W4A8;
# LN-fold consumer K limit; two-step q8 quantiser
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_spread
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_w8a8.py -m gpu -k "pingpong or lnf or w4a8_gemm or quantize or w8a8_stage" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -3 $o.tests.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 8192 --cfgs 57,64,100,101 --iters 30 > $o.gemm8192.log 2>&1 || exit 1
cat $o.gemm8192.log
timeout -k 10 300 python -u tools/bench_gemm.py --m 65536 --cfgs 57,64,100,101 --iters 10 > $o.gemm65536.log 2>&1 || exit 1
cat $o.gemm65536.log
timeout -k 10 400 python -u tools/bench_cfg_ab.py 2 8 "spread:qkv=100,proj=101,lin1=100,lin2=101;spread57:qkv=100,proj=100,lin1=100,lin2=100" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
