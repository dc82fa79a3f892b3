#!/bin/bash
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, one rocprofv3 --pmc pass each, no traces) of the eager
# bench step for every mode -> gpurun_out/pmc_<mode>.json (copy into profiles/ as
# r2_pmc_traffic_<mode>.json: bench.py reads the GEMM bytes per launch from it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for mode in w4a16 w4a8 w8a8; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_${mode}_$(echo $c | tr A-Z a-z | cut -d_ -f1)
    rm -rf "$d"
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$d" -o run -- \
      python3 bench.py --mode $mode --steps 2 --warmup 1 --no-cpu-baseline --no-graph > "$d.log" 2>&1 \
      || { echo "pmc pass $mode $c failed rc=$?"; tail -20 "$d.log"; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${mode}_fetch gpurun_out/pmc_${mode}_write > gpurun_out/pmc_$mode.json || exit 1
  echo "pmc $mode done"
done
