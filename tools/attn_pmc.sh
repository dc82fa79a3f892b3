# PMC passes over the attention micro-benchmark (one counter group per run, each under its own limit)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_attn -o p1 -- python3 tools/bench_attn.py --iters 2 > gpurun_out/pmc_attn1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o p2 -- python3 tools/bench_attn.py --iters 2 > gpurun_out/pmc_attn2.log 2>&1 || exit 1
