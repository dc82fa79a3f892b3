#!/bin/bash
# round 4: A&S 7.1.28 GELU in the int8 epilogues (exact-code tests + bench A/B), and the W4A8 shapes
# on int8-expanded weights (BF_W8 kernels, no unpack) vs the W4 ping-pong (cfg 86)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_q
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w8a8.py tests/test_w4a8.py -m gpu -k "stage_local or gemm" -s > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
grep -E "GELU|passed|failed" $o.tests.log | tail -12
timeout -k 10 200 python -u tools/bench_i8.py --m 16384 --cfgs 86 --iters 10 > $o.w4.log 2>&1 || { tail -20 $o.w4.log; exit 1; }
cat $o.w4.log
timeout -k 10 200 python -u tools/bench_i8.py --w8-vith --m 16384 --cfgs 81,82,83 --iters 10 > $o.w8.log 2>&1 || { tail -20 $o.w8.log; exit 1; }
cat $o.w8.log
for r in 1 2; do
  for lib in tools/ab/libsamq_pre_gelu.so new; do
    if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
    timeout -k 10 300 python -u bench.py --mode w4a8 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated > $o.b48.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w4a8 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b48.$r.$(basename $lib).log)"
  done
done
