# occupancy counters of the attention microbench (two PMC passes, each under its own limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc MeanOccupancyPerActiveCU --output-format csv -d gpurun_out/pmc_occ -o p1 -- python3 tools/bench_attn.py --iters 2 --batch 2 --window-only > gpurun_out/pmc_occ1.log 2>&1 || exit 1
SAMQ_LIB=$PWD/sam-quantization_amd/build_ab/attention_old.so timeout -s KILL 90 rocprofv3 --pmc MeanOccupancyPerActiveCU --output-format csv -d gpurun_out/pmc_occ_old -o p1 -- python3 tools/bench_attn.py --iters 2 --batch 2 --window-only > gpurun_out/pmc_occ2.log 2>&1 || exit 1
