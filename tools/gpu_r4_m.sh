#!/bin/bash
# round 4: exact-code tests (packed int8 quantiser, 24-bit row sums), global attention loop changes
# (ones region, exp2 ahead of the max, rotating slots) + variants A/B and timeline, window
# unscaled-Q A/B, cfg 111 (transposed f16 epilogue staging) tests + in-graph A/B, bench vs previous
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_m
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w8a8.py tests/test_w4a8.py tests/test_gpu_kernels.py -m gpu -k "w8a8 or stage_local or w4a8_gemm or layernorm or rel_attention or quantize or (pingpong and 111) or persistent_matches" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
SAMQ_LIB=tuning timeout -k 10 200 python -u tools/attn_variant_ab.py 0,512,128,32,64,256,288,16 2 8 > $o.gvar.log 2>&1 || { tail -20 $o.gvar.log; exit 1; }
cat $o.gvar.log
SAMQ_LIB=tools/ab/libsamq_prev.so timeout -k 10 120 python -u tools/attn_variant_ab.py 0 2 6 > $o.gprev.log 2>&1 || { tail -20 $o.gprev.log; exit 1; }
cat $o.gprev.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 0,8 2 1 > $o.tl.log 2>&1 || { tail -20 $o.tl.log; exit 1; }
tail -9 $o.tl.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 0,1 2 1 > $o.st.log 2>&1 || { tail -20 $o.st.log; exit 1; }
grep stamps $o.st.log | tail -1
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/win_variant_ab.py 0,1 6 > $o.win.log 2>&1 || { tail -20 $o.win.log; exit 1; }
cat $o.win.log
timeout -k 10 300 python -u tools/bench_cfg_ab.py 2 6 "f16t:qkv=111,lin1=111;f16tq:qkv=111;f16tl:lin1=111" > $o.ab111.log 2>&1 || { tail -20 $o.ab111.log; exit 1; }
cat $o.ab111.log
for lib in tools/ab/libsamq_prev.so new; do
  if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
  for m in w4a16 w4a8 w8a8; do
    st=20; [ $m = w4a8 ] && st=10
    timeout -k 10 300 python -u bench.py --mode $m --steps $st --warmup 3 --no-cpu-baseline --no-isolated > $o.b.$m.$(basename $lib).log 2>&1 || exit 1
    echo "$m $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b.$m.$(basename $lib).log)"
  done
done
