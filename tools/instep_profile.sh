#!/bin/bash
# rocprofv3 kernel trace of bench.py's timed configuration (graph replays with the timed lanes, no
# live roofline passes) -> profiles/instep_<mode>_b<imgs/launch>_l<lanes>_<source hash>.csv, the
# file bench.py reads its in-step GEMM roofline from.  usage: tools/instep_profile.sh [w4a16|w4a8]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mode=${1:-w4a16}
d=gpurun_out/instep_$mode
rm -rf "$d"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- \
  python3 bench.py --mode "$mode" --steps 10 --warmup 3 --no-cpu-baseline --no-isolated > "$d.log" 2>&1
name=$(python3 - "$mode" <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
line = [l for l in open(f"gpurun_out/instep_{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
c = d["config"]
print(f"instep_{sys.argv[1]}_b{c['per_gpu_batch'] // c['lanes']}_l{c['lanes']}_{bench.source_hash()}.csv")
PY
)
cp "$d/run_kernel_stats.csv" "gpurun_out/$name"
echo "in-step profile: gpurun_out/$name (copy into profiles/)"
