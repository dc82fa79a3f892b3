#!/bin/bash
# round 4: W4A8 in-graph upper bounds (timing-only): int8 GEMM epilogues, attention kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_j
SAMQ_LIB=tuning timeout -k 10 600 python -u tools/bench_cfg_ab_w4a8.py 2 4 "noepi:qkv=94,proj=94,lin1=94,lin2=94;noepi_q8g:lin1=94;noattn:skip_win=1,skip_glob=1;noglob:skip_glob=1" > $o.ab48.log 2>&1 || exit 1
cat $o.ab48.log
