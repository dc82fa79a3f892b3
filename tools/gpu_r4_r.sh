#!/bin/bash
# round 4: A&S 7.1.28 GELU in the W4A16 ping-pong epilogue: encoder tests + bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_r
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_kernels.py -m gpu -k "encoder or vith or (pingpong and gelu) or lanes or config4" -s > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
grep -E "parity|max-abs|passed|failed" $o.tests.log | tail -12
for r in 1 2 3; do
  for lib in tools/ab/libsamq_pre_gelu16.so new; do
    if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $o.b16.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w4a16 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b16.$r.$(basename $lib).log)"
  done
done
