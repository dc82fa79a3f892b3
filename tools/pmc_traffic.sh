#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (MI355X_MICROARCH.md §HBM): one rocprofv3
# pass per counter (FETCH_SIZE and WRITE_SIZE do not fit one pass), --pmc only (no traces).
# usage: tools/pmc_traffic.sh [bench args...]   -> gpurun_out/pmc_fetch/, gpurun_out/pmc_write/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${*:-"--steps 2 --warmup 1 --no-cpu-baseline --no-graph"}
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 bench.py $ARGS \
    > $d.log 2>&1 || { echo "pmc pass $c failed rc=$?"; tail -20 $d.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write
