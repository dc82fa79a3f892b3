#!/bin/bash
# same-box A/B of bench.py (W4A16 default config) over (library, extra args) pairs, alternated:
#   tools/gpu_ab3.sh "<lib|product>:<args>" ...      e.g. "product:" "product:--no-fold-ln" "build_ab/x.so:"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2 3; do
  for spec in "$@"; do
    lib=${spec%%:*}; args=${spec#*:}
    if [ "$lib" = product ]; then unset SAMQ_LIB; else export SAMQ_LIB=$PWD/sam-quantization_amd/$lib; fi
    echo -n "[$spec] "
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated $args 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
unset SAMQ_LIB
