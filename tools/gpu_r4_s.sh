#!/bin/bash
# round 4: softmax numerator table in the W8A8 (fq_vit) attention kernels: exact-code tests + bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_s
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w8a8.py tests/test_gpu_kernels.py -m gpu -k "w8a8 or q8" -s > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
grep -E "attention|codes|passed|failed" $o.tests.log | tail -14
for r in 1 2 3; do
  for lib in tools/ab/libsamq_pre_ptab.so new; do
    if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
    timeout -k 10 300 python -u bench.py --mode w8a8 --steps 30 --warmup 5 --no-cpu-baseline --no-isolated > $o.b88.$r.$(basename $lib).log 2>&1 || exit 1
    echo "w8a8 $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b88.$r.$(basename $lib).log)"
  done
done
