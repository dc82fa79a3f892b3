#!/bin/bash
# same-box A/B: W4A16 bench with the LayerNorm fold on / off, alternated
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in "--fold-ln" ""; do
    echo -n "fold[$v]: "; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated $v "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
