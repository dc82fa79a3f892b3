#!/bin/bash
# round 4: in-graph upper bounds of the non-GEMM kernels (timing-only: LayerNorms / window /
# global attention left out of the W4A16 graph)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_h
timeout -k 10 500 python -u tools/bench_cfg_ab.py 2 6 "noln:skip_ln=1;nowin:skip_win=1;noglob:skip_glob=1;noattn:skip_win=1,skip_glob=1" > $o.ab.log 2>&1 || exit 1
cat $o.ab.log
