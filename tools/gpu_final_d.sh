#!/bin/bash
# round-end: the three bench lines of the final build once more (box-to-box spread check)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in w4a16 w4a8 w8a8; do
  st=20; [ $m = w4a8 ] && st=10
  timeout -k 10 300 python bench.py --mode $m --steps $st --warmup 5 --no-cpu-baseline > gpurun_out/r4d_bench_$m.log 2>&1 || exit 1
  echo "$m $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/r4d_bench_$m.log)"
done
