#!/bin/bash
# round 4: unscaled-Q window attention as the product default (tests), global attention with the
# DMA moved into group 1's VALU segment (G1DMA) A/B + stamps, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_n
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w4a8.py tests/test_gpu_kernels.py -m gpu -k "stage_local or rel_attention or vith_vs_oracle" -s > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
grep -E "off by one|passed|failed" $o.tests.log | tail -30
SAMQ_LIB=tuning timeout -k 10 200 python -u tools/attn_variant_ab.py 0,1024,1280,256 2 8 > $o.gvar.log 2>&1 || { tail -20 $o.gvar.log; exit 1; }
cat $o.gvar.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 1024,1032 2 1 > $o.tl.log 2>&1 || { tail -20 $o.tl.log; exit 1; }
tail -9 $o.tl.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 1024,1025 2 1 > $o.st.log 2>&1 || { tail -20 $o.st.log; exit 1; }
grep stamps $o.st.log | tail -1
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/win_variant_ab.py 0,2 6 > $o.win.log 2>&1 || { tail -20 $o.win.log; exit 1; }
cat $o.win.log
for m in w4a16 w4a8; do
  st=20; [ $m = w4a8 ] && st=10
  timeout -k 10 300 python -u bench.py --mode $m --steps $st --warmup 3 --no-cpu-baseline --no-isolated > $o.b.$m.log 2>&1 || exit 1
  echo "$m $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('parity'))" $o.b.$m.log)"
done
