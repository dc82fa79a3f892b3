# bench.py (W4A16 default config, no CPU leg / isolated pass) over variant libraries, alternated twice:
#   tools/bench_variants.sh build_ab/a.so build_ab/b.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    echo -n "$lib: "; SAMQ_LIB=$PWD/sam-quantization_amd/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
