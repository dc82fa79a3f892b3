# window + global attention microbench over variant libraries: tools/attn_variants_all.sh build_ab/a.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    echo "$lib: "; SAMQ_LIB=$PWD/sam-quantization_amd/$lib timeout -k 10 120 python tools/bench_attn.py --batch 2 --iters 20 2>&1 | grep "attention" || exit 1
  done
done
