#!/bin/bash
# Round-end evidence on one GPU box: GPU suite, smoke, the three bench lines (with CPU baselines),
# in-step traces of every mode (+ W4A16 B=8 / 4 lanes and G=128), PMC HBM traffic passes.
# Each step under its own time limit; a crash / abort / timeout ends the session.
#   tools/final_round.sh <tag>      -> gpurun_out/<tag>_*.log, gpurun_out/instep_*.json, gpurun_out/pmc_*.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-final}
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== [$name] $(date +%T) start"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "=== [$name] $(date +%T) rc=$rc"
  tail -n 3 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
run gputests 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu -rA
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_w4a16 400 python bench.py --steps 20 --warmup 5
run bench_w4a8 400 python bench.py --mode w4a8 --steps 10 --warmup 3
run bench_w8a8 400 python bench.py --mode w8a8 --steps 20 --warmup 5
run bench_g128 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --groupsize 128
run instep16 500 bash tools/instep_profile.sh w4a16
run instep48 500 bash tools/instep_profile.sh w4a8
run instep88 500 bash tools/instep_profile.sh w8a8
run instepb8 500 bash tools/instep_profile.sh w4a16 --batch 8
run instepg 500 bash tools/instep_profile.sh w4a16 --groupsize 128
run pmc 900 bash tools/pmc_all.sh
# keep the summaries only (gpurun copies back at most 64 MiB of gpurun_out/)
rm -rf gpurun_out/instep_*_/ gpurun_out/pmc_*_fetch gpurun_out/pmc_*_write
du -sh gpurun_out
exit 0
