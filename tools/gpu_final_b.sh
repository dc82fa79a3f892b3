#!/bin/bash
# round-end evidence, part B: in-step kernel traces of every bench mode (+ G = 128), PMC HBM traffic,
# attention PMC counters -- for the build whose source hash bench.py looks up in profiles/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r4b}
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== [$name] $(date +%T) start"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "=== [$name] $(date +%T) rc=$rc"
  tail -n 2 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
run instep16 300 bash tools/instep_profile.sh w4a16
run instep48 300 bash tools/instep_profile.sh w4a8
run instep88 300 bash tools/instep_profile.sh w8a8
run instepg 300 bash tools/instep_profile.sh w4a16 --groupsize 128
run attnpmc 200 bash tools/attn_pmc.sh 2
run pmc 600 bash tools/pmc_all.sh
rm -rf gpurun_out/instep_*_/ gpurun_out/pmc_*_fetch gpurun_out/pmc_*_write gpurun_out/pmc_attn
du -sh gpurun_out
exit 0
