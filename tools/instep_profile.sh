#!/bin/bash
# rocprofv3 kernel trace of bench.py's timed configuration (graph replays with the timed lanes, no
# live roofline passes); the dispatches inside bench's roctx "samq_timed_steps" range ->
# gpurun_out/instep_<mode>_b<imgs/launch>_l<lanes>_<source hash>.json (copy into profiles/: bench.py
# reads its in-step GEMM roofline from it), plus the whole-run --stats summary next to it.
# usage: tools/instep_profile.sh [w4a16|w4a8|w8a8] [extra bench.py args, e.g. --batch 8]
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mode=${1:-w4a16}
shift || true
steps=10
tag=$(echo "$*" | tr -c 'a-zA-Z0-9' '_')
d=gpurun_out/instep_$mode$tag
rm -rf "$d"
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d "$d" -o run --output-format csv -- \
  python3 bench.py --mode "$mode" --steps $steps --warmup 3 --no-cpu-baseline --no-isolated --no-modes "$@" > "$d.log" 2>&1
name=$(python3 - "$mode" "$d.log" <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
c = d["config"]
print(bench.instep_name(sys.argv[1], c['per_gpu_batch'] // c['lanes'], c['lanes'], c.get('groupsize', -1)))
PY
)
python3 tools/instep_window.py "$d" $steps "gpurun_out/$name.json" "$mode"
cp "$d/run_kernel_stats.csv" "gpurun_out/${name}_wholerun_stats.csv"
echo "in-step profile: gpurun_out/$name.json (copy into profiles/)"
