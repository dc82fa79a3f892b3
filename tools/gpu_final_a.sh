#!/bin/bash
# round-end evidence, part A: the whole GPU suite, smoke, the three bench lines (with CPU baselines)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4final}
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== [$name] $(date +%T) start"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "=== [$name] $(date +%T) rc=$rc"
  tail -n 3 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
run gputests 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu -rfE
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench_w4a16 300 python bench.py --steps 20 --warmup 5
run bench_w4a8 300 python bench.py --mode w4a8 --steps 10 --warmup 3
run bench_w8a8 300 python bench.py --mode w8a8 --steps 20 --warmup 5
exit 0
