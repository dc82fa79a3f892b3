# PMC passes over the attention micro-benchmark (one counter group per run, each under its own limit)
# usage: bash tools/attn_pmc.sh [batch]   -> gpurun_out/pmc_attn/, summary gpurun_out/pmc_attn.txt
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
B=${1:-2}
rm -rf gpurun_out/pmc_attn
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_attn -o p1 -- python3 tools/bench_attn.py --iters 2 --batch $B > gpurun_out/pmc_attn1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o p2 -- python3 tools/bench_attn.py --iters 2 --batch $B > gpurun_out/pmc_attn2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc_attn -o p3 -- python3 tools/bench_attn.py --iters 2 --batch $B > gpurun_out/pmc_attn3.log 2>&1 || exit 1
python3 tools/pmc_kernel_counters.py gpurun_out/pmc_attn > gpurun_out/pmc_attn.txt
