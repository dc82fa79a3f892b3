set -e
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${VARS:-0 1 2 4}; do
  echo "VAR $v"; SAMQ_LIB=tuning SAMQ_WIN_VAR=$v timeout -k 10 120 python tools/bench_attn.py --batch 2 --iters 5 2>&1 | grep -E "attention window=14|stamps" | tail -2
done
