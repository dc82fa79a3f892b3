#!/bin/bash
# round 4: two-workgroups-per-CU GEMM tiles (v3 128x256, 4 waves of 128x64: cfg 25) in the graph --
# one workgroup's epilogue beside the other's main loop
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_i
timeout -k 10 300 python -u tools/bench_gemm.py --m 8192 --cfgs 57,64,25,22 --iters 30 > $o.g8192.log 2>&1 || exit 1
cat $o.g8192.log
timeout -k 10 600 python -u tools/bench_cfg_ab.py 2 6 "v25:qkv=25,proj=25,lin1=25,lin2=25;v25f16:qkv=25,lin1=25;v25res:proj=25,lin2=25;v22res:proj=22,lin2=22" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
SAMQ_LIB=tuning timeout -k 10 300 python -u tools/attn_variant_ab.py 0,8 2 8 > $o.attn.log 2>&1 || exit 1
cat $o.attn.log
