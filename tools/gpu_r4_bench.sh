#!/bin/bash
# round 4: bench lines (W4A16 with CPU baseline + parity stanza, W4A8 with parity, W8A8)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_bench
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $o.w4a16.log 2>&1 || { tail -30 $o.w4a16.log; exit 1; }
tail -1 $o.w4a16.log
timeout -k 10 500 python -u bench.py --mode w4a8 --steps 10 --warmup 3 > $o.w4a8.log 2>&1 || { tail -30 $o.w4a8.log; exit 1; }
tail -1 $o.w4a8.log
timeout -k 10 400 python -u bench.py --mode w8a8 --steps 20 --warmup 5 --no-cpu-baseline > $o.w8a8.log 2>&1 || { tail -30 $o.w8a8.log; exit 1; }
tail -1 $o.w8a8.log
