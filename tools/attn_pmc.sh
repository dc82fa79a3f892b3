cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k "attention" > gpurun_out/attn_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/attn_tests.log
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/bench_attn.log 2>&1; echo "bench rc=$?"; cat gpurun_out/bench_attn.log | grep attention
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn -o p1 -- python3 tools/bench_attn.py --iters 2 > gpurun_out/pmc_attn1.log 2>&1; echo "pmc rc=$?"
