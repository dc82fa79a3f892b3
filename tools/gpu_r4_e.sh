#!/bin/bash
# round 4: what the f16 epilogue (qkv, lin1+GELU) costs: stores vs math vs staging (timing-only cfgs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_e
SAMQ_LIB=tuning timeout -k 10 300 python -u tools/bench_gemm.py --m 65536 --cfgs 57,102,105,106 --iters 10 --shapes qkv,lin1 > $o.iso.log 2>&1 || exit 1
cat $o.iso.log
SAMQ_LIB=tuning timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 6 "noepi_f16:qkv=102,lin1=102;nostore:qkv=105,lin1=105;nomath:qkv=106,lin1=106" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
