#!/bin/bash
# round 4: hi + lo P in the window kernel's int8 store (W4A8): stage-local codes + cost (isolated and
# in the W4A8 step, tuning build SAMQ_ATTN_WIN=3 = without); global attention offset-MFMA and
# static-priority variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w4a8.py tests/test_gpu_kernels.py -m gpu -k "stage_local or rel_attention" -s > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
grep -E "attention|attn q8|passed|failed" $o.tests.log | tail -20
SAMQ_LIB=tuning timeout -k 10 150 python -u tools/win_variant_ab.py 0,3 6 > $o.win.log 2>&1 || { tail -20 $o.win.log; exit 1; }
cat $o.win.log
SAMQ_LIB=tuning timeout -k 10 250 python -u tools/attn_variant_ab.py 0,256,2048,2304 2 10 > $o.gvar.log 2>&1 || { tail -20 $o.gvar.log; exit 1; }
cat $o.gvar.log
SAMQ_LIB=tuning timeout -k 10 120 python -u tools/attn_variant_ab.py 256,257 2 1 > $o.st.log 2>&1 || { tail -20 $o.st.log; exit 1; }
grep stamps $o.st.log | tail -1
for r in 1 2; do
  for v in 0 3; do
    SAMQ_LIB=tuning SAMQ_ATTN_WIN=$v timeout -k 10 300 python -u bench.py --mode w4a8 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated > $o.b48.$v.$r.log 2>&1 || exit 1
    echo "w4a8 win=$v $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b48.$v.$r.log)"
  done
done
