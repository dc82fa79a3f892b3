#!/bin/bash
# round 4: exact-code tests for the packed int8 quantiser + offset-in-C global attention, bench
# A/B vs the previous build, window-attention unscaled-Q variant A/B, global-attention timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w8a8.py tests/test_w4a8.py tests/test_gpu_kernels.py -m gpu -k "w8a8 or w4a8 or layernorm or rel_attention or quantize" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/win_variant_ab.py 0,1 6 > $o.win.log 2>&1 || { tail -20 $o.win.log; exit 1; }
cat $o.win.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 0,8 2 1 > $o.tl.log 2>&1 || { tail -20 $o.tl.log; exit 1; }
tail -9 $o.tl.log
SAMQ_LIB=tools/ab/libsamq_prev.so timeout -k 10 120 python -u tools/attn_variant_ab.py 0 2 6 > $o.gprev.log 2>&1 || { tail -20 $o.gprev.log; exit 1; }
cat $o.gprev.log
SAMQ_LIB=tuning timeout -k 10 200 python -u tools/attn_variant_ab.py 0,512,128,32,64,256,288,16 2 8 > $o.gvar.log 2>&1 || { tail -20 $o.gvar.log; exit 1; }
cat $o.gvar.log
for r in 1; do
  for lib in tools/ab/libsamq_prev.so new; do
    if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
    timeout -k 10 300 python -u bench.py --mode w4a8 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated > $o.b48.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w4a8 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b48.$r.$(basename $lib).log)"
    timeout -k 10 300 python -u bench.py --mode w8a8 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $o.b88.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w8a8 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b88.$r.$(basename $lib).log)"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $o.b16.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w4a16 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b16.$r.$(basename $lib).log)"
  done
done
