#!/bin/bash
# round 4: W4A16 lane-stagger sweep on the final kernels (interleaved, two rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for st in -1 1 2 4; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-isolated --lane-stagger=$st > gpurun_out/r4_u.$st.$r.log 2>&1 || exit 1
    echo "stagger $st $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/r4_u.$st.$r.log)"
  done
done
