# A/B of the attention kernels: samq/libsamq_hip_tuning.so (A, built by hand from another
# attention.hip) vs the product library (B), same process order alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  echo "A:"; SAMQ_LIB=tuning timeout -k 10 120 python tools/bench_attn.py --batch 2 --iters 20 2>&1 | grep attention || exit 1
  echo "B:"; timeout -k 10 120 python tools/bench_attn.py --batch 2 --iters 20 2>&1 | grep attention || exit 1
done
